"""Pin the CPU oracle (oracle/cista_oracle.py) to golden vectors produced by the REAL reference
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import fixtures as fx
from oracle.cista_oracle import CistaLSTCOracle, conv3x3, softshrink, upsample_bilinear2x
from tests.conftest import rel_err

TOL32 = 2e-6     # oracle fp32 vs reference fp32 frames (different GEMM order)
TOLST = 5e-5     # states under the expansive "stress" init amplify fp32 reduction-order noise
TOL64 = 1e-12    # oracle fp64 vs reference fp64


def default_params():
    sd = torch.load(fx_path("f1_default.pth.tar"), weights_only=True)["state_dict"]
    return fx.collapse_tied({k: v.numpy() for k, v in sd.items()}, 5)


def fx_path(name):
    import os
    from tests.conftest import GOLDEN
    return os.path.join(GOLDEN, name)


@pytest.mark.parametrize("tag", ["default", "stress"])
def test_f1_sequence(golden, tag):
    d = golden("f1_64x64.npz")
    params = default_params() if tag == "default" else fx.stress_params(64, 5, 5)
    recs, st = CistaLSTCOracle(params, 5, np.float32).run_sequence(d["voxels"])
    for f in range(3):
        assert rel_err(recs[f], d[f"{tag}_rec{f}"]) < TOL32
    for k, v in zip(["c_lstc", "z", "h", "c"], [st[0], st[1], st[2][0], st[2][1]]):
        assert rel_err(v, d[f"{tag}_state_{k}"]) < TOLST, k
    recs64, _ = CistaLSTCOracle(params, 5, np.float64).run_sequence(d["voxels"])
    for f in range(3):
        assert np.abs(recs64[f] - d[f"{tag}_rec{f}_f64"]).max() < TOL64


def test_f1_intermediates(golden):
    d = golden("f1_64x64.npz")
    o = CistaLSTCOracle(fx.stress_params(64, 5, 5), 5, np.float32)
    st0 = [d["stress_state0_c_lstc"], d["stress_state0_z"],
           (d["stress_state0_h"], d["stress_state0_c"])]
    tr = {}
    o.forward(d["voxels"][1], d["stress_rec0"], st0, trace=tr)
    assert rel_err(tr["x1"][0], d["inter_x1"][0]) < TOL32
    assert rel_err(tr["c_lstc"][0], d["inter_c_lstc"][0]) < TOL32
    for i in range(5):
        assert rel_err(tr["ista"][i][0], (list(d["inter_ista_z_in"][1:]) + [d["inter_z_final"][0]])[i]) < TOLST
    for k in ("dg_y", "h", "c", "u", "pre_sigmoid"):
        assert rel_err(tr[k][0], d[f"inter_{k}"][0]) < TOLST, k


def test_f2_c32_depth2(golden):
    d = golden("f2_32x48_c32_d2.npz")
    recs, st = CistaLSTCOracle(fx.stress_params(32, 2, 5, seed=11), 2).run_sequence(d["voxels"])
    for f in range(4):
        assert rel_err(recs[f], d[f"rec{f}"]) < TOL32
    assert rel_err(st[1], d["state_z"]) < TOLST


def test_f4_drift(golden):
    d = golden("f4_64x64_seq15.npz")
    recs, _ = CistaLSTCOracle(fx.stress_params(64, 5, 5)).run_sequence(d["voxels"])
    assert rel_err(recs, d["rec"]) < 1e-5
    assert rel_err(d["rec"], d["rec_f64"]) < 1e-5      # fp32 reference drift vs truth


@pytest.mark.slow
def test_f3_full_size(golden):
    d = golden("f3_180x240.npz")
    recs, st = CistaLSTCOracle(fx.stress_params(64, 5, 5)).run_sequence(d["voxels"])
    for f in range(2):
        assert rel_err(recs[f], d[f"rec{f}"]) < TOL32
    z = st[1]
    assert abs(z.astype(np.float64).sum() - d["state1_z_sum"]) <= 1e-4 * d["state1_z_abssum"]


def test_voxelizer_matches_reference(golden):
    d = golden("vox_180x240.npz")
    raw = fx.voxelize(d["events"], 5, 240, 180)
    np.testing.assert_array_equal(raw, d["voxel_raw"])
    np.testing.assert_array_equal(fx.normalize_voxel(raw), d["voxel"])


def test_voxelizer_spill_matches_reference(golden):
    """Out-of-frame events that the reference's np.add.at adds to another pixel / bin (x >= W,
    y >= H, negative x, a negative index wrapping to the grid's end): the restatement reproduces
    the reference's own grids (tests/golden/make_golden_spill.py) bit for bit."""
    d = golden("vox_spill.npz")
    for k in range(4):
        nb, H, W = (int(v) for v in d[f"shape_{k}"])
        ev = d[f"events_{k}"]
        outside = (ev[:, 1] <= -1) | (ev[:, 1] >= W) | (ev[:, 2] <= -1) | (ev[:, 2] >= H)
        assert outside.sum() >= 90
        got = fx.voxelize(ev, nb, W, H)
        assert np.array_equal(got.view(np.uint32), d[f"np_{k}"].view(np.uint32)), k


def test_primitives_vs_torch():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 6, 9, 11)).astype(np.float32)
    w = rng.standard_normal((4, 6, 3, 3)).astype(np.float32)
    b = rng.standard_normal(4).astype(np.float32)
    for stride in (1, 2):
        conv = torch.nn.Conv2d(6, 4, 3, stride, 1, padding_mode="reflect")
        conv.weight.data[:] = torch.from_numpy(w)
        conv.bias.data[:] = torch.from_numpy(b)
        ref = conv(torch.from_numpy(x)).detach().numpy()
        assert np.abs(conv3x3(x, w, b, stride) - ref).max() < 1e-5
    up = torch.nn.functional.interpolate(torch.from_numpy(x), size=[18, 22], mode="bilinear",
                                         align_corners=False).numpy()
    assert np.abs(upsample_bilinear2x(x) - up).max() < 1e-6
    # softshrink formula with a NEGATIVE lambda differs from F.softshrink
    lam = np.float32(-0.3)
    v = np.array([-1.0, -0.1, 0.0, 0.2, 1.0], np.float32)
    np.testing.assert_allclose(softshrink(v, lam),
                               np.maximum(v - lam, 0) - np.maximum(-v - lam, 0))


def test_stress_recipe_is_deterministic():
    a = fx.stress_params(64, 5, 5)
    b = fx.stress_params(64, 5, 5)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    assert [k for k, _ in fx.param_shapes()] == list(a.keys())


def test_ssim_oracle_properties():
    """oracle/ssim_oracle.py (parity unpinned: pytorch_msssim is absent): identical images give
    1, the fp32 and fp64 restatements agree, and the window is the normalised 11-tap Gaussian."""
    from oracle import ssim_oracle as so
    g = np.random.default_rng(0)
    Y = g.uniform(0, 1, (2, 1, 40, 48))
    X = np.clip(Y + g.normal(0, 0.1, Y.shape), 0, 1)
    assert abs(so.ssim(Y, Y) - 1.0) < 1e-12
    s64 = so.ssim(X, Y)
    s32 = so.ssim(X.astype(np.float32), Y.astype(np.float32))
    assert 0.0 < s64 < 1.0 and abs(s32 - s64) < 1e-5
    w = so.gauss_1d()
    assert w.shape == (11,) and abs(float(w.sum()) - 1.0) < 1e-6 and np.argmax(w) == 5


def test_v2e_oracle_properties():
    """oracle/v2e_oracle.py (parity unpinned): lin_log's two branches, no events from a static
    scene in the deterministic configuration, and ON/OFF events with the right sign."""
    from oracle import v2e_oracle as vo
    x = np.array([0.0, 10.0, 20.0, 100.0], np.float32)
    np.testing.assert_allclose(vo.lin_log(x), [0.0, 10 * np.log(20) / 20, np.log(20), np.log(100)], rtol=1e-7)
    det = dict(sigma_thres=0.0, leak_rate_hz=0.0, shot_noise_rate_hz=0.0)
    static = np.full((1, 5, 8, 8), 100.0, np.float32)
    vox, n = vo.V2EOracle(**det).forward(static, np.linspace(0, 0.04, 5)[None])
    assert n == 0 and not vox.any()
    ramp = np.stack([np.full((8, 8), 30.0 * (1.3 ** k), np.float32) for k in range(5)])[None]
    vox, n = vo.V2EOracle(**det).forward(ramp, np.linspace(0, 0.04, 5)[None])
    assert n > 0 and vox.min() >= 0 and vox.max() > 0            # brightening: ON events only
    vox, _ = vo.V2EOracle(**det).forward(ramp[:, ::-1].copy(), np.linspace(0, 0.04, 5)[None])
    assert vox.max() <= 0 and vox.min() < 0


@pytest.mark.parametrize("tag", ["default", "stress"])
def test_torch_cpu_restatement_f1(golden, tag):
    """The PyTorch-CPU restatement (bench.py's cpu_baseline leg) against the same vectors."""
    from oracle.cista_oracle_torch import CistaLSTCTorchCPU
    d = golden("f1_64x64.npz")
    params = default_params() if tag == "default" else fx.stress_params(64, 5, 5)
    recs, st = CistaLSTCTorchCPU(params, 5).run_sequence(d["voxels"])
    for f in range(3):
        assert rel_err(recs[f], d[f"{tag}_rec{f}"]) < TOL32
    for k, v in zip(["c_lstc", "z", "h", "c"], [st[0], st[1], st[2][0], st[2][1]]):
        assert rel_err(v, d[f"{tag}_state_{k}"]) < TOLST, k
    recs64, _ = CistaLSTCTorchCPU(params, 5, torch.float64).run_sequence(d["voxels"])
    for f in range(3):
        assert np.abs(recs64[f] - d[f"{tag}_rec{f}_f64"]).max() < TOL64


def test_torch_cpu_restatement_f2(golden):
    from oracle.cista_oracle_torch import CistaLSTCTorchCPU
    d = golden("f2_32x48_c32_d2.npz")
    recs, st = CistaLSTCTorchCPU(fx.stress_params(32, 2, 5, seed=11), 2).run_sequence(d["voxels"])
    for f in range(4):
        assert rel_err(recs[f], d[f"rec{f}"]) < TOL32
    assert rel_err(st[1], d["state_z"]) < TOLST
