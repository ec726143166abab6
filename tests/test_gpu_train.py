"""BPTT backward of the HIP path against gradients produced by the
real reference's autograd on CPU (tests/golden/make_golden_grads.py).

Bars (max|hip - ref| / max|ref| per gradient tensor):
  * 32x48 fixtures (g1, g2): GTOL = 2e-4 against the fp32 reference.  The reference's own fp32
    gradients differ from its fp64 gradients by up to 4.8e-5 there (stored as *_noise32_*) and
    the HIP gradients measured 4.8e-5 on MI355X, so the bar is ~4x either;
  * c3 size (180x240, 15 frames, grads_180x240_seq15.npz): the fp32 reference itself is up to
    2.3e-3 from the fp64 truth (the recurrence amplifies rounding), so the HIP gradients are held
    against the fp64 truth: err(hip, f64) <= max(4 x err(ref fp32, f64), 5e-4) per tensor.  Any
    fp32 rounding pattern lands at a random point of the same amplified spread: two HIP builds
    differing only in the rounding of the bilinear staging measured 1.3e-3 and 2.4e-3 on We (ref
    fp32 2.3e-3), and 3.6e-4 on the upsample weights, whose fp32-reference error happened to be
    1.1e-4.  A BPTT bug shows up orders of magnitude above this (the 32x48 fixtures hold the tight
    2e-4 bar where the reference's own noise is 5e-5).
The forward outputs keep the 1e-4 bar.
"""
import numpy as np
import pytest
import torch

from oracle import fixtures as fx
from tests.conftest import rel_err
from v2e2v_amd import CistaLSTCNet

pytestmark = pytest.mark.gpu
DEV = "cuda"
GTOL = 2e-4


def model(C=64, depth=5):
    m = CistaLSTCNet([32, 48], base_channels=C, depth=depth, num_bins=5)
    params = fx.stress_params(C, depth, 5, seed=21, lam=0.05)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, depth)
    m.load_state_dict(sd, strict=True)
    return m.to(DEV)


def grads_by_name(m):
    out = {}
    for k, p in m.named_parameters():
        out[k.replace("lista_blocks.0.", "lista.")] = p.grad.detach().cpu().numpy()
    return out


def gpu(x, rg=False):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV).requires_grad_(rg)


def test_one_frame_all_gradients(golden):
    d = golden("grads_32x48.npz")
    m = model()
    leaves = [gpu(d["g1_prev_image"], True)] + [gpu(d[f"g1_prev_{n}"], True) for n in ("c_lstc", "z", "h", "c")]
    ev = gpu(d["voxels"][1], True)                   # the events' gradient (We dgrad) too
    rec, st = m(ev, leaves[0], [leaves[1], leaves[2], (leaves[3], leaves[4])])
    outs = [rec, st[0], st[1], st[2][0], st[2][1]]
    loss = sum((o * gpu(d[f"g1_R{i}"])).sum() for i, o in enumerate(outs))
    loss.backward()
    torch.cuda.synchronize()
    bad = {}
    for k, g in grads_by_name(m).items():
        e = rel_err(g, d[f"g1_f32_param_{k}"])
        if not e < GTOL:
            bad[k] = e
    for i, n in enumerate(["prev_image", "c_lstc", "z", "h", "c"]):
        e = rel_err(leaves[i].grad.detach().cpu().numpy(), d[f"g1_f32_grad_{n}"])
        if not e < GTOL:
            bad["input:" + n] = e
    e = rel_err(ev.grad.detach().cpu().numpy(), d["g1_f32_grad_events"])
    if not e < GTOL:
        bad["input:events"] = e
    assert not bad, bad


def test_three_frame_bptt_l1(golden):
    """train_e2v.py:108-120: prev_img = output.clone() (no detach), states carried, L1 loss on
    the last frame, one backward through all frames."""
    d = golden("grads_32x48.npz")
    m = model()
    B, _, H, W = d["g2_target"].shape
    prev = torch.zeros(B, 1, H, W, device=DEV)
    state = None
    for s in range(3):
        out, state = m(gpu(d["voxels"][s]), prev, state)
        prev = out.clone()
    loss = torch.nn.functional.l1_loss(out, gpu(d["g2_target"]))
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - float(d["g2_f32_loss"])) <= 1e-4 * abs(float(d["g2_f32_loss"]))
    bad = {}
    for k, g in grads_by_name(m).items():
        e = rel_err(g, d[f"g2_f32_param_{k}"])
        if not e < GTOL:
            bad[k] = e
    assert not bad, bad


def test_gradient_accumulation_across_sequences(golden):
    """The frames reach the parameters through one flat conduit tensor per parameter version
    (CistaLSTCNet._grad_conduit), dropped once its gradient is computed.  Two sequences
    backpropagated one after the other without an optimizer step accumulate gA + gB; both
    forwarded first and backpropagated through one summed loss give the same; a forward with
    grad enabled and no backward changes nothing."""
    d = golden("grads_32x48.npz")
    m = model()
    B, _, H, W = d["g2_target"].shape
    tgt = gpu(d["g2_target"])

    def seq(order):
        prev = torch.zeros(B, 1, H, W, device=DEV)
        state = None
        for s in order:
            out, state = m(gpu(d["voxels"][s]), prev, state)
            prev = out.clone()
        return torch.nn.functional.l1_loss(out, tgt)

    def grads():
        torch.cuda.synchronize()
        return {k: p.grad.detach().clone() for k, p in m.named_parameters()}

    m.zero_grad(set_to_none=True)
    seq([0, 1, 2]).backward()
    ga = grads()
    m.zero_grad(set_to_none=True)
    seq([2, 1, 0]).backward()
    gb = grads()
    m.zero_grad(set_to_none=True)
    seq([1, 0]).sum()                                  # forward with grad, never backpropagated
    seq([0, 1, 2]).backward()
    seq([2, 1, 0]).backward()
    acc = grads()
    m.zero_grad(set_to_none=True)
    (seq([0, 1, 2]) + seq([2, 1, 0])).backward()
    joint = grads()
    for k in ga:
        want = (ga[k] + gb[k]).cpu().numpy()
        assert rel_err(acc[k].cpu().numpy(), want) < 1e-6, k
        assert rel_err(joint[k].cpu().numpy(), want) < 1e-5, k
        assert acc[k].shape == dict(m.named_parameters())[k].shape


def test_training_forward_equals_inference_forward(golden):
    d = golden("grads_32x48.npz")
    m = model()
    ev = gpu(d["voxels"][0])
    prev = torch.zeros(2, 1, 32, 48, device=DEV)
    with torch.no_grad():
        r0, s0 = m(ev, prev, None)
    r1, s1 = m(ev, prev, None)                      # grad mode: the training kernels
    assert r1.requires_grad
    assert torch.equal(r0, r1.detach())
    for a, b in zip([s0[0], s0[1], s0[2][0], s0[2][1]], [s1[0], s1[1], s1[2][0], s1[2][1]]):
        assert torch.equal(a, b.detach())


def test_report_gradient_errors(golden, capsys):
    """Not a bar: prints the measured gradient errors next to the reference's own fp32 noise."""
    d = golden("grads_32x48.npz")
    m = model()
    B, _, H, W = d["g2_target"].shape
    prev = torch.zeros(B, 1, H, W, device=DEV)
    state = None
    for s in range(3):
        out, state = m(gpu(d["voxels"][s]), prev, state)
        prev = out.clone()
    torch.nn.functional.l1_loss(out, gpu(d["g2_target"])).backward()
    rows = [(k, rel_err(g, d[f"g2_f32_param_{k}"]), float(d[f"g2_noise32_param_{k}"]))
            for k, g in grads_by_name(m).items()]
    with capsys.disabled():
        for k, e, n in sorted(rows, key=lambda r: -r[1])[:6]:
            print(f"\n  grad {k:40s} hip-vs-ref32 {e:.2e}   ref32-vs-ref64 {n:.2e}", end="")
        print()


def test_c3_size_bptt_against_fp64_truth(golden):
    """Config c3's frame size and sequence length (train_e2v.py:108-130): 180x240, 15 frames,
    prev_img = output.clone(), L1 on the last frame, one backward through the sequence."""
    from tests.golden.g3_spec import G3, g3_inputs, g3_params
    d = golden("grads_180x240_seq15.npz")
    vox, target = g3_inputs()
    assert float(vox.astype(np.float64).sum()) == float(d["vox_sum"])     # same inputs as the generator
    c = G3
    m = CistaLSTCNet([c["H"], c["W"]], base_channels=c["C"], depth=c["depth"], num_bins=5)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in g3_params().items()}, c["depth"])
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    prev = torch.zeros(c["B"], 1, c["H"], c["W"], device=DEV)
    state = None
    for s in range(c["L"]):
        out, state = m(gpu(vox[s]), prev, state)
        prev = out.clone()
    loss = torch.nn.functional.l1_loss(out, gpu(target))
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(out.detach().cpu().numpy(), d["f32_last_frame"]) < 1e-4
    assert abs(loss.item() - float(d["f64_loss"])) <= 1e-4 * abs(float(d["f64_loss"]))
    bad, rows = {}, []
    for k, g in grads_by_name(m).items():
        e = rel_err(g, d[f"f64_param_{k}"])
        bar = max(4 * float(d[f"noise32_param_{k}"]), 5e-4)
        rows.append((k, e, float(d[f"noise32_param_{k}"])))
        if not e <= bar:
            bad[k] = (e, bar)
    print("\n" + "\n".join(f"  c3 grad {k:40s} hip-vs-f64 {e:.2e}   ref32-vs-f64 {n:.2e}"
                            for k, e, n in sorted(rows, key=lambda r: -r[1])[:6]))
    assert not bad, bad


def test_c3_batch8_bptt_against_fp64_truth(golden):
    """BASELINE config c3's batch (and c4's per-rank shape): 180x240, B=8, 5 frames of
    train_e2v.py:108-130.  The split-wgrad partial sums are split over the B x tiles pixel tiles
    (cista_backward.hpp wgrad_split_kernel), so their grid depends on B: g1/g2 pin B <= 2 only."""
    from tests.golden.g4_spec import G4, g4_inputs, g4_params
    d = golden("grads_180x240_b8.npz")
    vox, target = g4_inputs()
    assert float(vox.astype(np.float64).sum()) == float(d["vox_sum"])     # same inputs as the generator
    c = G4
    m = CistaLSTCNet([c["H"], c["W"]], base_channels=c["C"], depth=c["depth"], num_bins=5)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in g4_params().items()}, c["depth"])
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    prev = torch.zeros(c["B"], 1, c["H"], c["W"], device=DEV)
    state = None
    for s in range(c["L"]):
        out, state = m(gpu(vox[s]), prev, state)
        prev = out.clone()
    loss = torch.nn.functional.l1_loss(out, gpu(target))
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(out.detach().cpu().numpy(), d["f32_last_frame"]) < 1e-4
    assert abs(loss.item() - float(d["f64_loss"])) <= 1e-4 * abs(float(d["f64_loss"]))
    bad, rows = {}, []
    for k, g in grads_by_name(m).items():
        e = rel_err(g, d[f"f64_param_{k}"])
        bar = max(4 * float(d[f"noise32_param_{k}"]), 5e-4)
        rows.append((k, e, float(d[f"noise32_param_{k}"])))
        if not e <= bar:
            bad[k] = (e, bar)
    print("\n" + "\n".join(f"  c3 B=8 grad {k:40s} hip-vs-f64 {e:.2e}   ref32-vs-f64 {n:.2e}"
                            for k, e, n in sorted(rows, key=lambda r: -r[1])[:6]))
    assert not bad, bad


@pytest.mark.parametrize("xscale", [1.0, 3.0e5])
def test_wgrad_tr_kernel_matches_fp64(xscale):
    """The split-f16 weight-gradient kernel on its own (the backward's stacked ISTA P launch,
    cista_wgrad_ista_p: wgrad_tr_kernel + reduce_partials_kernel) against an fp64 conv weight
    gradient over the reflect-padded input: dW = sum_P G(P) x Xpad(P + t), db = sum_P G(P).
    xscale = 3e5 puts the activations beyond the fp16 hi part, so every tile takes the re-staging
    path with a power-of-two pre-scale (X has no per-tensor scale); the bar stays fp32-level."""
    import ctypes
    from v2e2v_amd import _lib
    C, D, B, H, W = 64, 5, 2, 36, 52              # ragged tiles: 18 x 26 half-res, 6 x 16 tiles
    h, w = H // 2, W // 2
    m = CistaLSTCNet([H, W], base_channels=C, depth=D, num_bins=5).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(5)
    G = torch.rand(D * B, h, w, 2 * C, device=DEV, generator=g) * 2 - 1
    X = (torch.rand(D * B, h, w, C, device=DEV, generator=g) * 2 - 1) * xscale
    sc = torch.tensor([8192.0, 1.0 / 8192.0], device=DEV)        # max |G s| <= 16384
    dW = torch.empty(2 * C, C, 3, 3, device=DEV)
    db = torch.empty(2 * C, device=DEV)
    ws = m.train_workspace(B, H, W, DEV)
    L = _lib.lib()
    cfg = m._cfg()
    _lib.check(L.cista_wgrad_ista_p(ctypes.byref(cfg), B, H, W, G.data_ptr(), X.data_ptr(), sc.data_ptr(),
                                    dW.data_ptr(), db.data_ptr(), ws.data_ptr(), ws.numel(),
                                    torch.cuda.current_stream().cuda_stream), "cista_wgrad_ista_p")
    torch.cuda.synchronize()
    Gd = G.double().permute(0, 3, 1, 2)
    Xd = torch.nn.functional.pad(X.double().permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect")
    ref = torch.nn.grad.conv2d_weight(Xd, (2 * C, C, 3, 3), Gd)
    # fp32 accumulation over 4680 pixels: ~sqrt(N) x 6e-8 of the largest entry
    assert rel_err(dW.double().cpu().numpy(), ref.cpu().numpy()) < 1e-5
    assert rel_err(db.double().cpu().numpy(), Gd.sum((0, 2, 3)).cpu().numpy()) < 1e-5


@pytest.mark.parametrize("xscale", [1.0, 3.0e5])
def test_wgrad_tr_s2_kernel_matches_fp64(xscale):
    """W0's stride-2 weight gradient (cista_wgrad_w0: wgrad_tr_kernel<XS_S2> over a parity-split
    5 x 33 halo + reduce_partials_kernel) against an fp64 stride-2 conv weight gradient over the
    reflect-padded input.  36 x 52 gives 18 x 26 outputs: ragged 2 x 16 tiles in x and the
    reflected bottom / right halo rows; xscale = 3e5 sends every tile through the re-staging path."""
    import ctypes
    from v2e2v_amd import _lib
    C, B, H, W = 64, 3, 36, 52
    h, w = H // 2, W // 2
    m = CistaLSTCNet([H, W], base_channels=C, depth=2, num_bins=5).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(6)
    G = torch.rand(B, h, w, C, device=DEV, generator=g) * 2 - 1
    X = (torch.rand(B, H, W, C, device=DEV, generator=g) * 2 - 1) * xscale
    sc = torch.tensor([8192.0, 1.0 / 8192.0], device=DEV)
    dW = torch.empty(C, C, 3, 3, device=DEV)
    db = torch.empty(C, device=DEV)
    ws = m.train_workspace(B, H, W, DEV)
    L = _lib.lib()
    cfg = m._cfg()
    _lib.check(L.cista_wgrad_w0(ctypes.byref(cfg), B, H, W, G.data_ptr(), X.data_ptr(), sc.data_ptr(),
                                dW.data_ptr(), db.data_ptr(), ws.data_ptr(), ws.numel(),
                                torch.cuda.current_stream().cuda_stream), "cista_wgrad_w0")
    torch.cuda.synchronize()
    Gd = G.double().permute(0, 3, 1, 2)
    Xd = torch.nn.functional.pad(X.double().permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect")
    ref = torch.nn.grad.conv2d_weight(Xd, (C, C, 3, 3), Gd, stride=2)
    assert rel_err(dW.double().cpu().numpy(), ref.cpu().numpy()) < 1e-5
    assert rel_err(db.double().cpu().numpy(), Gd.sum((0, 2, 3)).cpu().numpy()) < 1e-5


@pytest.mark.parametrize("stride", [1, 2])
def test_wgrad_tr_outlier_tiles_then_o1_tiles(stride):
    """A split of the split-f16 wgrad walks its tiles in order with a per-tile X pre-scale: a tile
    whose X holds 1e12 outliers is re-staged at 2^-26, and the O(1) tiles the same split walks after
    it must be staged unscaled again (at 2^-26 an O(1) value is below the smallest fp16 subnormal
    and vanishes).  The outlier tiles have G = 0, so they add nothing and the expected gradient is
    O(1); fp64 conv weight gradient as the truth.  Stride 1: the stacked ISTA P launch (the first
    tile of every split is one of sample 0's, all outlier tiles); stride 2: W0 at 180 x 240, B = 2
    (3 tiles per split, the first from sample 0's top 60 output rows)."""
    import ctypes
    from v2e2v_amd import _lib
    C = 64
    L = _lib.lib()
    g = torch.Generator(device=DEV).manual_seed(8)
    if stride == 1:
        D, B, H, W = 5, 2, 180, 240
        h, w = H // 2, W // 2
        m = CistaLSTCNet([H, W], base_channels=C, depth=D, num_bins=5).to(DEV)
        G = torch.rand(D * B, h, w, 2 * C, device=DEV, generator=g) * 2 - 1
        X = torch.rand(D * B, h, w, C, device=DEV, generator=g) * 2 - 1
        G[0] = 0.0
        X[0, ::7, ::9, ::5] = 1e12
        dW = torch.empty(2 * C, C, 3, 3, device=DEV)
        db = torch.empty(2 * C, device=DEV)
        fn, args = L.cista_wgrad_ista_p, (dW, db)
    else:
        B, H, W = 2, 180, 240
        h, w = H // 2, W // 2
        m = CistaLSTCNet([H, W], base_channels=C, depth=2, num_bins=5).to(DEV)
        G = torch.rand(B, h, w, C, device=DEV, generator=g) * 2 - 1
        X = torch.rand(B, H, W, C, device=DEV, generator=g) * 2 - 1
        G[0, :60] = 0.0
        X[0, 2:100:7, ::9, ::5] = 1e12          # read only by output rows <= 50 (G = 0 there)
        dW = torch.empty(C, C, 3, 3, device=DEV)
        db = torch.empty(C, device=DEV)
        fn = L.cista_wgrad_w0
    sc = torch.tensor([8192.0, 1.0 / 8192.0], device=DEV)
    ws = m.train_workspace(B, H, W, DEV)
    _lib.check(fn(ctypes.byref(m._cfg()), B, H, W, G.data_ptr(), X.data_ptr(), sc.data_ptr(), dW.data_ptr(),
                  db.data_ptr(), ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream), "wgrad")
    torch.cuda.synchronize()
    Gd = G.double().permute(0, 3, 1, 2)
    Xd = torch.nn.functional.pad(X.double().permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect")
    ref = torch.nn.grad.conv2d_weight(Xd, tuple(dW.shape), Gd, stride=stride)
    assert float(ref.abs().max()) < 1e4                  # the outliers contribute nothing
    assert rel_err(dW.double().cpu().numpy(), ref.cpu().numpy()) < 1e-5
    assert rel_err(db.double().cpu().numpy(), Gd.sum((0, 2, 3)).cpu().numpy()) < 1e-5


@pytest.mark.parametrize("H,W,C,NB", [(6, 8, 32, 5), (8, 12, 32, 5), (12, 10, 32, 5), (12, 16, 96, 5), (10, 14, 128, 5),
                                      (8, 8, 256, 5), (16, 20, 64, 1), (12, 16, 32, 8), (14, 18, 64, 3)])
def test_small_images_bptt_against_fp64_autograd(H, W, C, NB):
    """The dgrads fold the reflect padding in their epilogue (EPI_FOLD + fold_fix_kernel) when the
    half-resolution input has rows 1 and n-2 distinct (h, w >= 4) and take the padded-domain
    dgrad + fold_reflect_kernel pass otherwise: 6x8 (h = 3, the pass), 8x12 (h = 4, the smallest
    epilogue fold, every border row and column a reflected one) and 12x10 (w = 5).  Two-frame
    BPTT (prev_img = output.clone(), states carried, L1 on the last frame) against fp64 autograd
    through the PyTorch-CPU restatement of the reference forward.  C = 96, 128 and 256 (the largest training supports) cover the
    training path beyond the reference default's channel counts (any multiple of 32)."""
    from oracle.cista_oracle_torch import CistaLSTCTorchCPU
    depth, B = 2, 2
    params = fx.stress_params(C, depth, NB, seed=H * 100 + W, lam=0.05)
    m = CistaLSTCNet([H, W], base_channels=C, depth=depth, num_bins=NB)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, depth)
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    rng = np.random.default_rng(H * W)
    vox = rng.standard_normal((2, B, NB, H, W)).astype(np.float32)
    target = rng.random((B, 1, H, W)).astype(np.float32)
    prev, state = torch.zeros(B, 1, H, W, device=DEV), None
    for f in range(2):
        out, state = m(gpu(vox[f]), prev, state)
        prev = out.clone()
    torch.nn.functional.l1_loss(out, gpu(target)).backward()
    torch.cuda.synchronize()
    o = CistaLSTCTorchCPU(params, depth, dtype=torch.float64, requires_grad=True)
    prev_t, st_t = torch.zeros(B, 1, H, W, dtype=torch.float64), None
    for f in range(2):
        out_t, st_t = o.forward_grad(torch.from_numpy(vox[f]).double(), prev_t, st_t)
        prev_t = out_t.clone()
    torch.nn.functional.l1_loss(out_t, torch.from_numpy(target).double()).backward()
    bad = {}
    for k, g in grads_by_name(m).items():
        e = rel_err(g, o.p[k].grad.numpy())
        if not e < GTOL:
            bad[k] = e
    assert not bad, bad


def test_training_two_region_tiling_equals_single():
    """Training at a batch whose forward convs take the two-region tiling (B=40 at 180x240:
    2400 items for the 192-pixel convs, past plan_tiles' 1024) while B=1 keeps one region: the
    training forward's frame and states of every checked sample equal its own B=1 training run
    bit for bit; the events / previous-image gradients of one backward (fed by the saved
    activations the split-tile SV kernels wrote) agree within 1e-5 of their max: the backward's
    fp16 gradient splits take one power-of-two scale per batch tensor, so a sample's small
    values meet the fp16 subnormals at a different point in a batch than alone (last bits)."""
    B = 40
    m = CistaLSTCNet([180, 240], base_channels=64, depth=5, num_bins=5)
    params = fx.stress_params(64, 5, 5, seed=41, lam=0.05)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, 5)
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    rng = np.random.default_rng(5)
    vox = rng.standard_normal((B, 5, 180, 240)).astype(np.float32)
    prev = rng.random((B, 1, 180, 240)).astype(np.float32)
    ev, pi = gpu(vox, True), gpu(prev, True)
    r, s = m(ev, pi, None)
    (r.sum() + s[1].square().mean()).backward()
    for i in (0, 23, B - 1):
        evi, pii = gpu(vox[i:i + 1], True), gpu(prev[i:i + 1], True)
        ri, si = m(evi, pii, None)
        assert torch.equal(r[i:i + 1].detach(), ri.detach()), i
        assert torch.equal(s[1][i:i + 1].detach(), si[1].detach()), i
        assert torch.equal(s[2][1][i:i + 1].detach(), si[2][1].detach()), i
        # the state term's mean over B (vs over 1) scales its gradient by 1 / B: use the same loss
        (ri.sum() + si[1].square().sum() / s[1].numel()).backward()
        e1, e2 = rel_err(ev.grad[i:i + 1].cpu().numpy(), evi.grad.cpu().numpy()), \
            rel_err(pi.grad[i:i + 1].cpu().numpy(), pii.grad.cpu().numpy())
        print(f"sample {i}: events grad {e1:.2e}, prev-image grad {e2:.2e}")
        assert e1 < 1e-5 and e2 < 1e-5, (i, e1, e2)


@pytest.mark.parametrize("H,W,C,B", [(180, 240, 64, 8), (6, 8, 32, 2), (10, 14, 128, 2)])
def test_side_stream_wgrads_bit_identical(monkeypatch, H, W, C, B):
    """The backward's weight gradients run on a side stream beside the dgrad chain
    (cista_abi.hip on_side / join_side).  They are the same kernels on the same inputs, so a BPTT
    step (3 frames) gives bit-identical parameter and input gradients with the side stream on and
    off (CISTA_BWD_SIDE, read per call); a missed write-after-read hazard between the two streams
    would show up here as a differing value.  Shapes: config c3's (180x240, B=8; the folded
    dgrads with their scale tickets), 6x8 at C = 32 (half-res 3x4: the padded-domain dgrad +
    fold pass and scale_of launches) and 10x14 at C = 128 (other channel counts on both streams)."""
    L = 3
    m = CistaLSTCNet([H, W], base_channels=C, depth=5, num_bins=5)
    params = fx.stress_params(C, 5, 5, seed=43, lam=0.05)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, 5)
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    rng = np.random.default_rng(9)
    vox = rng.standard_normal((L, B, 5, H, W)).astype(np.float32)
    target = gpu(rng.random((B, 1, H, W)).astype(np.float32))

    def step(side):
        monkeypatch.setenv("CISTA_BWD_SIDE", "1" if side else "0")
        m.zero_grad(set_to_none=True)
        evs = [gpu(vox[f], True) for f in range(L)]
        prev, state = torch.zeros(B, 1, H, W, device=DEV), None
        for f in range(L):
            out, state = m(evs[f], prev, state)
            prev = out.clone()
        (out - target).abs().mean().backward()
        torch.cuda.synchronize()
        return grads_by_name(m), [e.grad.detach().cpu().numpy() for e in evs]

    g0, e0 = step(False)
    g1, e1 = step(True)
    g2, e2 = step(True)                                  # and repeatable
    for k in g0:
        assert np.array_equal(g0[k], g1[k]) and np.array_equal(g1[k], g2[k]), k
    for f in range(L):
        assert np.array_equal(e0[f], e1[f]) and np.array_equal(e1[f], e2[f]), f
