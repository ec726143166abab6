"""The emulator restatement's raw-event mode (oracle/v2e_oracle.py, reference
v2e/v2e_model.py:504-518,527-534) against its own voxel-grid mode: the same state machine, so
the raw rows scattered into voxels with the reference's voxel arithmetic (:477-502) must give the
voxel mode's grid bit for bit, and the rows must come out sorted by (b, t) with pixel-order ties.
Parity unpinned against the reference itself (its module imports cv2, absent here)."""
import numpy as np
import pytest

from oracle import v2e_oracle as vo

f32 = np.float32
DET = dict(sigma_thres=0.0, leak_rate_hz=0.0, shot_noise_rate_hz=0.0)


def video(B, F, H, W, seed=0, t0=0.0):
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(f32)
    bg = 40 + 30 * np.sin(xx / 5.0) * np.cos(yy / 7.0) + g.uniform(0, 5, (H, W))
    out = np.zeros((B, F, H, W), f32)
    for b in range(B):
        for f in range(F):
            cx, cy = 6 + 1.5 * (f + 0.3 * b) + 3 * t0, H / 2 + 3 * np.sin(0.3 * f + b)
            out[b, f] = np.clip(bg + 180 * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / 30.0), 0, 255)
    return out


def scatter(rows, B, nb, H, W):
    """The reference's voxel accumulation (:477-502) applied to raw rows in their order."""
    vox = np.zeros((B, nb, H, W), f32)
    t, x, y, p, b = (rows[:, k] for k in range(5))
    ti = np.floor(t).astype(f32)
    dts = (t - ti).astype(f32)
    vl = (p * (f32(1) - dts)).astype(f32)
    vr = (p * dts).astype(f32)
    bi, xi, yi, k = b.astype(np.int64), x.astype(np.int64), y.astype(np.int64), ti.astype(np.int64)
    # row by row, left cell then right cell: a cell's sum in the reference's (n, it) order
    right = (ti + 1) < nb
    two = lambda u, v: np.stack([u, v], 1).reshape(-1)
    keep = two(np.ones_like(right), right)
    idx = (two(bi, bi)[keep], two(k, k + 1)[keep], two(yi, yi)[keep], two(xi, xi)[keep])
    np.add.at(vox, idx, two(vl, vr)[keep])
    return vox


@pytest.mark.parametrize("extra", [{}, {"refractory_period_s": 0.004, "cutoff_hz": 15.0},
                                   {"pos_thres": 0.1, "neg_thres": 0.3}])
def test_raw_rows_rebuild_the_voxel_grid(extra):
    cfg = dict(DET, **extra)
    B, F, H, W, nb = 3, 6, 20, 28, 5
    grid, raw = vo.V2EOracle(**cfg), vo.V2EOracle(output_mode="raw", **cfg)
    for k in range(2):
        fr = video(B, F, H, W, seed=1, t0=k)
        tf = np.tile(0.15 * k + 0.01 * np.arange(F), (B, 1))
        vox, n = grid.forward(fr, tf)
        rows, m = raw.forward(fr, tf)
        assert n == m == rows.shape[0] > 0 and rows.dtype == f32 and rows.shape[1] == 5
        np.testing.assert_array_equal(scatter(rows, B, nb, H, W), vox)
        # sorted by b, then t; equal (b, t) in pixel order
        key = np.lexsort((rows[:, 1], rows[:, 2], rows[:, 0], rows[:, 4]))
        np.testing.assert_array_equal(key, np.arange(rows.shape[0]))
        assert set(np.unique(rows[:, 3])) <= {-1.0, 1.0} and (rows[:, 0] > 0).all()


def test_raw_static_video_is_a_1d_empty_tensor():
    """No frame step runs an iteration: the reference never concatenates and returns
    torch.tensor([]) (shape (0,), :347)."""
    fr = np.full((1, 4, 8, 8), 90.0, f32)
    rows, n = vo.V2EOracle(output_mode="raw", **DET).forward(fr, np.tile(0.01 * np.arange(4), (1, 1)))
    assert n == 0 and rows.shape == (0,)
