"""Parity of the HIP path (libcista_hip.so, called through the C ABI / the drop-in module)
against (a) golden vectors produced by the real reference and (b) the numpy oracle on seeded
inputs.  Bars (north_star: 1e-4 relative fp32; SURVEY section 7's parity metric): frames
elementwise, max |hip - ref| / |ref| <= 1e-4 per pixel (elem_rel_err); states, which hold exact
zeros, max |hip - ref| / max |ref| <= 1e-4 per tensor (rel_err).
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import fixtures as fx
from oracle.cista_oracle import CistaLSTCOracle
from tests.conftest import elem_rel_err, rel_err
from v2e2v_amd import CistaLSTCNet, _lib

pytestmark = pytest.mark.gpu
TOL = 1e-4
DEV = "cuda"


def make_model(C=64, depth=5, nb=5, params=None):
    m = CistaLSTCNet([64, 64], base_channels=C, depth=depth, num_bins=nb)
    if params is not None:
        sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()},
                            depth)
        m.load_state_dict(sd, strict=True)
    return m.to(DEV).eval()


def nhwc(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV).permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).cpu().numpy()


def gpu(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


def run_seq(model, voxels, prev=None):
    F_, B, nb, H, W = voxels.shape
    prev = torch.zeros(B, 1, H, W, device=DEV) if prev is None else prev
    states = None
    recs = []
    with torch.no_grad():
        for f in range(F_):
            prev, states = model(gpu(voxels[f]), prev, states)
            recs.append(prev.cpu().numpy())
    torch.cuda.synchronize()
    return np.stack(recs), [s.cpu().numpy() if not isinstance(s, tuple) else
                            tuple(t.cpu().numpy() for t in s) for s in states]


# ------------------------------------------------------------------ per-stage KATs (F1, frame 1)
@pytest.fixture(scope="module")
def f1_stage(golden):
    d = golden("f1_64x64.npz")
    m = make_model(params=fx.stress_params(64, 5, 5))
    packed = m.packed_params()
    ws = m.workspace(1, 64, 64, torch.device(DEV))
    cfg = _lib.CistaConfig(64, 5, 5)
    return d, m, packed, ws, cfg, _lib.lib()


def call(fn, *args):
    _lib.check(fn(*args), fn.__name__)
    torch.cuda.synchronize()


def test_stage_input(f1_stage):
    d, m, packed, ws, cfg, L = f1_stage
    x1 = torch.empty(1, 32, 32, 64, device=DEV)
    ev, img = gpu(d["voxels"][1][:1]), gpu(d["stress_rec0"][:1])   # keep alive across the call
    call(L.cista_stage_input, ctypes.byref(cfg), packed.data_ptr(), 1, 64, 64,
         ev.data_ptr(), img.data_ptr(), x1.data_ptr(), ws.data_ptr(), ws.numel(), None)
    assert rel_err(nchw(x1)[0], d["inter_x1"][0]) < TOL


def test_stage_lstc(f1_stage):
    d, m, packed, ws, cfg, L = f1_stage
    z = torch.empty(1, 32, 32, 128, device=DEV)
    c = torch.empty_like(z)
    x1 = nhwc(d["inter_x1"])
    zp, cp = nhwc(d["stress_state0_z"][:1]), nhwc(d["stress_state0_c_lstc"][:1])
    call(L.cista_stage_lstc, ctypes.byref(cfg), packed.data_ptr(), 1, 32, 32, x1.data_ptr(),
         zp.data_ptr(), cp.data_ptr(), z.data_ptr(), c.data_ptr(), ws.data_ptr(), ws.numel(), None)
    assert rel_err(nchw(c)[0], d["inter_c_lstc"][0]) < TOL
    assert rel_err(nchw(z)[0], d["inter_ista_z_in"][0]) < TOL


@pytest.mark.parametrize("iters", [1, 5])
def test_stage_ista(f1_stage, iters):
    d, m, packed, ws, cfg, L = f1_stage
    x1 = nhwc(d["inter_x1"])
    z = nhwc(d["inter_ista_z_in"][:1])
    call(L.cista_stage_ista, ctypes.byref(cfg), packed.data_ptr(), 1, 32, 32, x1.data_ptr(),
         z.data_ptr(), iters, ws.data_ptr(), ws.numel(), None)
    ref = d["inter_ista_z_in"][1] if iters == 1 else d["inter_z_final"][0]
    assert rel_err(nchw(z)[0], ref) < TOL


def test_stage_decoder(f1_stage):
    d, m, packed, ws, cfg, L = f1_stage
    z = nhwc(d["inter_z_final"])
    hp, cp = nhwc(d["stress_state0_h"][:1]), nhwc(d["stress_state0_c"][:1])
    h = torch.empty(1, 32, 32, 64, device=DEV)
    c = torch.empty_like(h)
    call(L.cista_stage_decoder, ctypes.byref(cfg), packed.data_ptr(), 1, 32, 32, z.data_ptr(),
         hp.data_ptr(), cp.data_ptr(), h.data_ptr(), c.data_ptr(), ws.data_ptr(), ws.numel(), None)
    assert rel_err(nchw(h)[0], d["inter_h"][0]) < TOL
    assert rel_err(nchw(c)[0], d["inter_c"][0]) < TOL


def test_stage_output(f1_stage):
    d, m, packed, ws, cfg, L = f1_stage
    hs = nhwc(d["inter_h"])
    rec = torch.empty(1, 1, 64, 64, device=DEV)
    pre = torch.empty_like(rec)
    call(L.cista_stage_output, ctypes.byref(cfg), packed.data_ptr(), 1, 32, 32, hs.data_ptr(),
         rec.data_ptr(), pre.data_ptr(), ws.data_ptr(), ws.numel(), None)
    assert rel_err(pre.cpu().numpy()[0], d["inter_pre_sigmoid"][0]) < TOL
    assert rel_err(rec.cpu().numpy()[0], d["stress_rec1"][0]) < TOL


# ------------------------------------------------------------------ whole-model golden sequences
@pytest.mark.parametrize("tag", ["default", "stress"])
def test_f1_sequence(golden, tag):
    d = golden("f1_64x64.npz")
    if tag == "default":
        ck = torch.load(__import__("os").path.join(__import__("tests.conftest", fromlist=["GOLDEN"]).GOLDEN,
                                                   "f1_default.pth.tar"), weights_only=True)
        m = CistaLSTCNet([64, 64]).to(DEV).eval()
        m.load_state_dict(ck["state_dict"], strict=True)       # reference checkpoint layout
    else:
        m = make_model(params=fx.stress_params(64, 5, 5))
    recs, st = run_seq(m, d["voxels"])
    for f in range(3):
        assert rel_err(recs[f], d[f"{tag}_rec{f}"]) < TOL, f
        assert rel_err(recs[f], d[f"{tag}_rec{f}_f64"]) < TOL, f
        assert elem_rel_err(recs[f], d[f"{tag}_rec{f}"]) < TOL, f
        assert elem_rel_err(recs[f], d[f"{tag}_rec{f}_f64"]) < TOL, f
    for k, v in zip(["c_lstc", "z", "h", "c"], [st[0], st[1], st[2][0], st[2][1]]):
        assert rel_err(v, d[f"{tag}_state_{k}"]) < TOL, k


def test_f2_c32_depth2(golden):
    d = golden("f2_32x48_c32_d2.npz")
    m = make_model(C=32, depth=2, params=fx.stress_params(32, 2, 5, seed=11))
    recs, st = run_seq(m, d["voxels"])
    for f in range(4):
        assert rel_err(recs[f], d[f"rec{f}"]) < TOL
        assert elem_rel_err(recs[f], d[f"rec{f}"]) < TOL          # every pixel
    for k, v in zip(["c_lstc", "z", "h", "c"], [st[0], st[1], st[2][0], st[2][1]]):
        assert rel_err(v, d[f"state_{k}"]) < TOL, k


def test_f3_full_size(golden):
    d = golden("f3_180x240.npz")
    m = make_model(params=fx.stress_params(64, 5, 5))
    recs, st = run_seq(m, d["voxels"])
    for f in range(2):
        assert rel_err(recs[f], d[f"rec{f}"]) < TOL
        assert elem_rel_err(recs[f], d[f"rec{f}"]) < TOL
    for k, v in zip(["c_lstc", "z", "h", "c"], [st[0], st[1], st[2][0], st[2][1]]):
        row = v[0, :, v.shape[2] // 2, :]
        assert rel_err(row, d[f"state1_{k}_row"]) < TOL, k
        assert abs(v.astype(np.float64).sum() - d[f"state1_{k}_sum"]) <= TOL * d[f"state1_{k}_abssum"]


def test_f4_fifteen_frames(golden):
    d = golden("f4_64x64_seq15.npz")
    m = make_model(params=fx.stress_params(64, 5, 5))
    recs, _ = run_seq(m, d["voxels"])
    assert rel_err(recs, d["rec"]) < TOL
    assert rel_err(recs, d["rec_f64"]) < TOL
    assert elem_rel_err(recs, d["rec"]) < TOL
    assert elem_rel_err(recs, d["rec_f64"]) < TOL


def test_dark_frames_elementwise_vs_fp64():
    """Frames spanning 7.5e-7 .. 0.98 (final conv weights x30, bias -5): every pixel, the darkest
    included, within 1e-4 of its own fp64 value, over 3 recurrent frames.  The reference's own fp32
    path is at 2.3e-5 elementwise here (oracle fp32 vs fp64); pixels that dark are where an
    absolute (max-normalised) 1e-4 bar would hide a 100 % error."""
    p = fx.stress_params(64, 5, 5)
    p["final_conv.conv2d.weight"] = p["final_conv.conv2d.weight"] * np.float32(30)
    p["final_conv.conv2d.bias"] = p["final_conv.conv2d.bias"] - np.float32(5)
    vox = fx.synthetic_voxels(3, 2, 5, 64, 64, n_events=fx.density_matched_events(64, 64), seed=5)
    recs, _ = run_seq(make_model(params=p), vox)
    truth, _ = CistaLSTCOracle(p, 5, dtype=np.float64).run_sequence(vox)
    assert float(np.min(truth)) < 1e-5
    assert elem_rel_err(recs, truth) < TOL


# ------------------------------------------------------------------ oracle on seeded inputs
@pytest.mark.parametrize("C,depth,B,H,W", [(64, 5, 3, 36, 52), (64, 3, 2, 18, 30),
                                           (32, 1, 1, 4, 4), (64, 5, 1, 6, 8), (32, 2, 2, 50, 26),
                                           (96, 2, 2, 20, 28), (128, 2, 1, 16, 24)])
def test_oracle_random(C, depth, B, H, W):
    params = fx.stress_params(C, depth, 5, seed=100 + C + depth)
    vox = fx.synthetic_voxels(2, B, 5, H, W, n_events=max(8, fx.density_matched_events(H, W)),
                              seed=H * W)
    m = make_model(C=C, depth=depth, params=params)
    recs, st = run_seq(m, vox)
    o_recs, o_st = CistaLSTCOracle(params, depth).run_sequence(vox)
    assert rel_err(recs, o_recs) < TOL
    assert elem_rel_err(recs, o_recs) < TOL
    # every returned state (e2v_model.py:68-83): c_lstc, z, (h, c)
    for k, v, o in zip(["c_lstc", "z", "h", "c"], [st[0], st[1], st[2][0], st[2][1]],
                       [o_st[0], o_st[1], o_st[2][0], o_st[2][1]]):
        assert rel_err(v, o) < TOL, k


@pytest.mark.parametrize("nb,H,W", [(1, 10, 12), (3, 20, 14), (8, 8, 18), (9, 12, 10)])
def test_num_bins(nb, H, W):
    """Bin counts other than 5: the fused input stage + W0 (input_w0_kernel<NB>, 1..8 bins) and
    the unfused fallback (> 8 bins) against the oracle, with border rows/columns on every side."""
    params = fx.stress_params(32, 2, nb, seed=200 + nb)
    vox = fx.synthetic_voxels(2, 2, nb, H, W, n_events=max(8, fx.density_matched_events(H, W)),
                              seed=nb * 31 + H)
    m = make_model(C=32, depth=2, nb=nb, params=params)
    recs, st = run_seq(m, vox)
    o_recs, o_st = CistaLSTCOracle(params, 2).run_sequence(vox)
    assert rel_err(recs, o_recs) < TOL
    assert elem_rel_err(recs, o_recs) < TOL
    for k, v, o in zip(["c_lstc", "z", "h", "c"], [st[0], st[1], st[2][0], st[2][1]],
                       [o_st[0], o_st[1], o_st[2][0], o_st[2][1]]):
        assert rel_err(v, o) < TOL, k


def test_partial_none_states():
    """prev_states entries are None-able independently (reference e2v_model.py:68,82)."""
    params = fx.stress_params(64, 2, 5, seed=5)
    vox = fx.synthetic_voxels(2, 2, 5, 16, 24, n_events=60, seed=3)
    o = CistaLSTCOracle(params, 2)
    prev, st = o.forward(vox[0], np.zeros((2, 1, 16, 24), np.float32), None)
    mixed = [None, st[1], None]
    ref, ref_st = o.forward(vox[1], prev, mixed)
    m = make_model(C=64, depth=2, params=params)
    with torch.no_grad():
        rec, hst = m(gpu(vox[1]), gpu(prev), [None, gpu(st[1]), None])
    assert rel_err(rec.cpu().numpy(), ref) < TOL
    assert rel_err(hst[0].cpu().numpy(), ref_st[0]) < TOL


def test_states_layout_and_no_mutation():
    m = make_model(C=32, depth=1, params=fx.stress_params(32, 1, 5))
    vox = gpu(fx.synthetic_voxels(1, 2, 5, 16, 16, n_events=40)[0])
    prev = torch.rand(2, 1, 16, 16, device=DEV)
    with torch.no_grad():
        r1, s1 = m(vox, prev, None)
        keep = [s1[0].clone(), s1[1].clone(), s1[2][0].clone(), s1[2][1].clone()]
        vox_c, prev_c = vox.clone(), prev.clone()
        r2, s2 = m(vox, prev, s1)
        # NCHW states from a caller are accepted too
        r3, _ = m(vox, prev, [s1[0].contiguous(), s1[1].contiguous(),
                              (s1[2][0].contiguous(), s1[2][1].contiguous())])
    assert s1[1].shape == (2, 64, 8, 8) and s1[1].is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(vox, vox_c) and torch.equal(prev, prev_c)
    for a, b in zip(keep, [s1[0], s1[1], s1[2][0], s1[2][1]]):
        assert torch.equal(a, b)
    assert torch.equal(r2, r3)
    assert r1.shape == (2, 1, 16, 16) and float(r1.min()) > 0 and float(r1.max()) < 1


def test_alias_and_shape_errors():
    m = make_model(C=32, depth=1, params=fx.stress_params(32, 1, 5))
    with torch.no_grad(), pytest.raises(RuntimeError):
        m(torch.zeros(1, 5, 15, 16, device=DEV), torch.zeros(1, 1, 15, 16, device=DEV), None)
    with torch.no_grad(), pytest.raises(RuntimeError):
        m(torch.zeros(1, 4, 16, 16, device=DEV), torch.zeros(1, 1, 16, 16, device=DEV), None)
    packed = m.packed_params()
    ws = m.workspace(1, 16, 16, torch.device(DEV))
    ev = torch.zeros(1, 5, 16, 16, device=DEV)
    img = torch.zeros(1, 1, 16, 16, device=DEV)
    z = torch.zeros(1, 8, 8, 64, device=DEV)
    io = _lib.CistaFrameIO(ev.data_ptr(), img.data_ptr(), None, z.data_ptr(), None, None,
                           img.data_ptr(), z.data_ptr(), z.data_ptr(), z.data_ptr(), z.data_ptr())
    cfg = _lib.CistaConfig(32, 1, 5)
    st = _lib.lib().cista_forward(ctypes.byref(cfg), packed.data_ptr(), 1, 16, 16, ctypes.byref(io),
                                  ws.data_ptr(), ws.numel(), None)
    assert st == 5   # CISTA_ERR_ALIAS


def test_batch_equals_single_two_frames():
    """At B=12, 180x240 (720 workgroups per 128-column conv, more than are resident at once)
    every sample must equal its own B=1 run bit for bit, states included, over two recurrent
    frames: no cross-sample coupling anywhere in the frame schedule."""
    params = fx.stress_params(64, 5, 5, seed=21)
    m = make_model(params=params)
    B = 12
    rng = np.random.default_rng(5)
    vox = gpu(rng.standard_normal((2, B, 5, 180, 240)).astype(np.float32))
    prev = torch.rand(B, 1, 180, 240, device=DEV)
    with torch.no_grad():
        r, s = m(vox[0], prev, None)
        r, s = m(vox[1], r, s)
        for i in (0, 5, 11):
            ri, si = m(vox[0, i:i + 1], prev[i:i + 1], None)
            ri, si = m(vox[1, i:i + 1], ri, si)
            assert torch.equal(r[i:i + 1], ri), i
            assert torch.equal(s[0][i:i + 1], si[0]) and torch.equal(s[1][i:i + 1], si[1]), i
            assert torch.equal(s[2][0][i:i + 1], si[2][0]) and torch.equal(s[2][1][i:i + 1], si[2][1]), i


def test_batch48_equals_single():
    """At B=48 (past the B >= 32 switches of the input border pass and every throughput tiling;
    2880 (pixel tile, column block) items per 128-column conv, several dispatch rounds) every
    sample must equal its own B=1 run bit for bit over two frames.
    This test found the upsample border strips' 128-pixel configuration giving last-bit
    differences on the border pixels; the strips now use one configuration at every batch."""
    params = fx.stress_params(64, 5, 5, seed=33)
    m = make_model(params=params)
    B = 48
    rng = np.random.default_rng(9)
    vox = gpu(rng.standard_normal((2, B, 5, 180, 240)).astype(np.float32))
    prev = torch.rand(B, 1, 180, 240, device=DEV)
    with torch.no_grad():
        r, s = m(vox[0], prev, None)
        r, s = m(vox[1], r, s)
        for i in (0, 17, 47):
            ri, si = m(vox[0, i:i + 1], prev[i:i + 1], None)
            ri, si = m(vox[1, i:i + 1], ri, si)
            assert torch.equal(r[i:i + 1], ri), i
            assert torch.equal(s[0][i:i + 1], si[0]) and torch.equal(s[1][i:i + 1], si[1]), i
            assert torch.equal(s[2][0][i:i + 1], si[2][0]) and torch.equal(s[2][1][i:i + 1], si[2][1]), i


@pytest.mark.parametrize("H,W,B", [(120, 180, 72), (90, 120, 140), (128, 194, 32), (74, 166, 60)])
def test_two_region_tiling_equals_single(H, W, B):
    """Two-region conv tiling (plan_tiles, cista_abi.hip): at these batches the forward convs
    of the 60 x 90 / 45 x 60 / 64 x 97 / 37 x 83 internal grids run as an exact-width region
    plus a column strip (10 / 12 columns; at 64 x 97 a 1-column strip of 64 x 1 tiles, at
    37 x 83 strips of 37 x 3 and 19 x 5 tiles) in the same launch, while a B=1 run keeps one
    region.  Every checked
    sample of the batched frame equals its own B=1 run bit for bit (same per-pixel arithmetic,
    different tiles), and one matches the oracle."""
    params = fx.stress_params(64, 2, 5, seed=H)
    m = make_model(depth=2, params=params)
    rng = np.random.default_rng(W)
    vox = rng.standard_normal((B, 5, H, W)).astype(np.float32)
    prev = rng.random((B, 1, H, W)).astype(np.float32)
    with torch.no_grad():
        r, s = m(gpu(vox), gpu(prev), None)
        for i in (0, B // 2 + 1, B - 1):
            ri, si = m(gpu(vox[i:i + 1]), gpu(prev[i:i + 1]), None)
            assert torch.equal(r[i:i + 1], ri), i
            assert torch.equal(s[0][i:i + 1], si[0]) and torch.equal(s[1][i:i + 1], si[1]), i
            assert torch.equal(s[2][0][i:i + 1], si[2][0]) and torch.equal(s[2][1][i:i + 1], si[2][1]), i
    o_rec, o_st = CistaLSTCOracle(params, 2).forward(vox[B - 1:B], prev[B - 1:B], None)
    assert elem_rel_err(r[B - 1:B].cpu().numpy(), o_rec) < TOL
    assert rel_err(s[1][B - 1:B].cpu().numpy(), o_st[1]) < TOL


def test_determinism_and_batch_independence():
    """Size-independent properties at the bench size: bit-identical re-runs, and sample i of a
    batched launch equals the same sample run alone (no cross-sample coupling)."""
    params = fx.stress_params(64, 5, 5)
    m = make_model(params=params)
    B = 4
    vox = gpu(np.random.default_rng(0).standard_normal((B, 5, 180, 240)).astype(np.float32))
    prev = torch.rand(B, 1, 180, 240, device=DEV)
    with torch.no_grad():
        r1, s1 = m(vox, prev, None)
        r2, s2 = m(vox, prev, None)
        ra, sa = m(vox[2:3], prev[2:3], None)
    assert torch.equal(r1, r2) and torch.equal(s1[1], s2[1])
    assert torch.equal(r1[2:3], ra) and torch.equal(s1[2][1][2:3], sa[2][1])


@pytest.mark.parametrize("H,W", [(20, 300), (300, 20)])
def test_border_segments_and_corner_blocks(H, W):
    """The input stage's border pass (input_border_kernel): strips longer than one 128-pixel
    segment (w or h = 150) and corner workgroups covering 64 samples each (B = 130: blocks of 64,
    64, 2).  Every sample of the batched frame equals its own B=1 run bit for bit, and one sample
    matches the oracle."""
    params = fx.stress_params(32, 1, 5, seed=77)
    m = make_model(C=32, depth=1, params=params)
    B = 130
    rng = np.random.default_rng(H)
    vox = rng.standard_normal((B, 5, H, W)).astype(np.float32)
    prev = rng.random((B, 1, H, W)).astype(np.float32)
    with torch.no_grad():
        r, s = m(gpu(vox), gpu(prev), None)
        for i in (0, 63, 64, 129):
            ri, si = m(gpu(vox[i:i + 1]), gpu(prev[i:i + 1]), None)
            assert torch.equal(r[i:i + 1], ri), i
            assert torch.equal(s[1][i:i + 1], si[1]), i
    o_rec, o_st = CistaLSTCOracle(params, 1).forward(vox[129:130], prev[129:130], None)
    assert rel_err(r[129:130].cpu().numpy(), o_rec) < TOL
    assert rel_err(s[1][129:130].cpu().numpy(), o_st[1]) < TOL
