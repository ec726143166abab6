"""GPU event voxelizer against the reference's numpy path.

Bar: BIT-EXACT.  The golden fixture vox_180x240.npz was produced by the reference's own
events_to_voxel_grid / event_preprocess (tests/golden/make_golden.py); the oracle restatement
(oracle/fixtures.py voxelize / normalize_voxel, numpy) is pinned to it by
tests/test_oracle_golden.py::test_voxelizer_matches_reference and covers the other cases.
"""
import numpy as np
import pytest
import torch

from oracle import fixtures as fx
from v2e2v_amd import event_process as ep

pytestmark = pytest.mark.gpu


def ref_raw(ev, nb, W, H):
    return fx.voxelize(ev, nb, W, H)


def assert_bits(got, want):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else got
    np.testing.assert_array_equal(got, want)          # -0.0 == 0.0 is fine, NaN never expected


def test_golden_180x240_raw_and_std(golden):
    d = golden("vox_180x240.npz")
    raw = ep.events_to_voxel_grid(d["events"], 5, 240, 180)
    assert_bits(raw, d["voxel_raw"])
    norm = ep.event_preprocess(raw, filter_hot_pixel=True)
    assert_bits(norm, d["voxel"])
    fused = ep.events_to_voxel_batch([d["events"]], 5, 240, 180, mode="std", filter_hot_pixel=True)
    assert_bits(fused[0], d["voxel"])


def test_input_not_modified(golden):
    d = golden("vox_180x240.npz")
    ev = torch.from_numpy(d["events"].copy()).cuda()
    before = ev.clone()
    ep.events_to_voxel_grid(ev, 5, 240, 180)
    assert torch.equal(ev, before)


def _windows(rng, H, W, sizes, hot=False):
    out = []
    for n in sizes:
        ev = fx.synthetic_events(n, H, W, rng)
        if hot and n > 50:                      # one pixel with many events: order-sensitive sums
            ev[::3, 1] = 7
            ev[::3, 2] = 3
        out.append(ev)
    return out


@pytest.mark.parametrize("H,W,nb", [(64, 64, 5), (32, 48, 3), (180, 240, 5), (31, 17, 7)])
def test_batch_matches_oracle(H, W, nb):
    rng = np.random.default_rng(H * W + nb)
    sizes = [0, 1, 2, 500, 3000, 15000, 7]
    wins = _windows(rng, H, W, sizes, hot=True)
    got = ep.events_to_voxel_batch(wins, nb, W, H).cpu().numpy()
    for b, ev in enumerate(wins):
        assert_bits(got[b], ref_raw(ev, nb, W, H))
    for mode in ("std", "maxmin"):
        for filt in (False, True):
            got = ep.events_to_voxel_batch(wins, nb, W, H, mode=mode, filter_hot_pixel=filt).cpu().numpy()
            for b, ev in enumerate(wins):
                assert_bits(got[b], fx.normalize_voxel(ref_raw(ev, nb, W, H), filt, mode))


def test_edge_cases():
    H, W, nb = 20, 30, 5
    # all events at one timestamp (deltaT == 0 -> 1.0, reference :40-41), polarity given as -1/1
    ev0 = np.array([[0.5, 3, 4, 1], [0.5, 3, 4, -1], [0.5, 29, 19, 0], [0.5, 0, 0, 1]], np.float64)
    # fractional coordinates truncate toward zero (astype(np.uint)); x = W and y = H are inside
    # the flat grid: the reference adds them to other pixels / bins, and so does this build
    ev1 = np.array([[0.0, 2.7, 1.2, 1], [0.01, 29.99, 19.5, 0], [0.02, 30.0, 2, 1], [0.03, 1, 20, 1],
                    [0.04, -0.5, 3, 1], [0.05, 5, 5, 1]], np.float64)
    got = ep.events_to_voxel_batch([ev0, ev1], nb, W, H).cpu().numpy()
    assert_bits(got[0], ref_raw(ev0, nb, W, H))
    assert_bits(got[1], ref_raw(ev1, nb, W, H))
    got = ep.events_to_voxel_batch([ev0, ev1], nb, W, H, strict=False).cpu().numpy()   # no check
    assert_bits(got[1], ref_raw(ev1, nb, W, H))
    ev1_in = ev1[[0, 1, 4, 5]]
    assert not np.array_equal(ref_raw(ev1, nb, W, H), ref_raw(ev1_in, nb, W, H))      # they do land


@pytest.mark.parametrize("bad", ["negative_x", "beyond_grid", "last_bin_row_below"])
def test_out_of_grid_raises_like_reference(bad):
    """np.add.at on the flat index x + y W + bin H W (utils/event_process.py:53-58) raises
    IndexError once an index reaches the grid size; the GPU path raises there too (both the fused
    per-window path and, for a large frame, the global-sort path)."""
    nb = 5
    for H, W in ((20, 30), (520, 520)):          # 520 x 520 >= 2^18 pixels: the keys + hipCUB path
        ev = np.array([[0.0, 2, 3, 1], [0.01, 5, 5, 0], [0.02, 7, 1, 1], [0.04, 1, 1, 1]], np.float64)
        if bad == "negative_x":
            ev[0, 1:3] = (-(nb * H * W + 7.0), 0.0)   # np.uint wraps; as intp below -size
        elif bad == "beyond_grid":
            ev[2, 2] = H * nb + 3                # y far below the frame: past the last bin
        else:
            ev[3, 2] = H                         # last event -> last bin, one row below the frame
        with pytest.raises(IndexError):
            fx.voxelize(ev, nb, W, H)            # the reference's behaviour (oracle restatement)
        with pytest.raises(IndexError):
            ep.events_to_voxel_batch([ev], nb, W, H)
        ep.events_to_voxel_batch([ev], nb, W, H, strict=False)     # unchecked: the event is dropped
    # a negative x whose flat index stays inside [-size, size) lands elsewhere in the reference
    # (moved back a row, or counted from the end of the grid): a spill, reproduced bit for bit
    ev = np.array([[0.0, -3, 0, 1], [0.01, -3, 5, 0], [0.04, 1, 1, 1]], np.float64)
    assert_bits(ep.events_to_voxel_batch([ev], nb, 30, 20)[0].cpu().numpy(), fx.voxelize(ev, nb, 30, 20))


@pytest.mark.parametrize("torch_semantics", [False, True])
def test_spill_matches_reference(golden, torch_semantics):
    """Events outside the frame whose flat index stays inside the grid (x >= W, y >= H, negative
    x): the reference's np.add.at / index_add_ add them to the cell that index names, in event
    order with the cell's own events.  Against grids the reference itself produced
    (tests/golden/make_golden_spill.py): a 20 x 30 window (fused path), one whose negative index
    wraps to the end of the grid (numpy; the torch twin raises there), a 64 x 64 window of three
    sorted segments, and 520 x 520 (global-sort path) -- each alone and the small ones batched."""
    d = golden("vox_spill.npz")
    wins, shapes = [], []
    for k in range(4):
        nb, H, W = (int(v) for v in d[f"shape_{k}"])
        ev = d[f"events_{k}"]
        want = d[f"torch_{k}" if torch_semantics else f"np_{k}"]
        if torch_semantics and not int(d[f"torch_ok_{k}"]):
            with pytest.raises(IndexError):
                ep.events_to_voxel_batch([ev], nb, W, H, torch_semantics=True)
            continue
        got = ep.events_to_voxel_batch([ev], nb, W, H, torch_semantics=torch_semantics)[0].cpu().numpy()
        assert_bits(got, want)
        if H == 20:
            wins.append(ev)
            shapes.append(want)
    if len(wins) > 1:                     # per-window spill flags in one batched call
        got = ep.events_to_voxel_batch(wins, 5, 30, 20, torch_semantics=torch_semantics).cpu().numpy()
        for b, want in enumerate(shapes):
            assert_bits(got[b], want)


def test_preprocess_thresholds_and_batch_shapes():
    rng = np.random.default_rng(3)
    H, W, nb = 40, 56, 5
    wins = _windows(rng, H, W, [4000, 9000, 100])
    raw = ep.events_to_voxel_batch(wins, nb, W, H)
    raw[:, :, 5, 5] = 9.0                        # hot pixels above both thresholds
    raw[:, :, 6, 6] = 4.5                        # between 20/5 and 25/5
    ref = raw.cpu().numpy()
    got = ep.event_preprocess(raw, filter_hot_pixel=True).cpu().numpy()
    for b in range(3):
        assert_bits(got[b], fx.normalize_voxel(ref[b], True, "std", 25.0))
    # the torch twin: threshold 20 / num_bins and float32 statistics (oracle pinned to the
    # reference's own function by tests/test_oracle_v2e_golden.py)
    from oracle import v2e_oracle as vo
    from tests.conftest import rel_err
    got = ep.event_preprocess_pytorch(raw[1], filter_hot_pixel=True).cpu().numpy()
    want = vo.event_preprocess_pytorch(ref[1], "std", True)
    assert rel_err(got, want) < 2e-6 and np.array_equal(got == 0, want == 0)
    assert torch.equal(raw.cpu(), torch.from_numpy(ref))      # not modified


@pytest.mark.parametrize("H,W,sizes", [(64, 64, [40000, 16384, 16385, 3]), (180, 240, [33000, 15000])])
def test_multi_segment_windows(H, W, sizes):
    """Windows larger than one sorted segment of the fused per-window kernel (16384 events):
    their left contributions of every segment go first, then the right ones, in event order."""
    rng = np.random.default_rng(sum(sizes))
    nb = 5
    wins = _windows(rng, H, W, sizes, hot=True)
    got = ep.events_to_voxel_batch(wins, nb, W, H).cpu().numpy()
    for b, ev in enumerate(wins):
        assert_bits(got[b], ref_raw(ev, nb, W, H))
    got = ep.events_to_voxel_batch(wins, nb, W, H, mode="std", filter_hot_pixel=True).cpu().numpy()
    for b, ev in enumerate(wins):
        assert_bits(got[b], fx.normalize_voxel(ref_raw(ev, nb, W, H), True, "std"))


def test_large_frame_many_events():
    """720x1280 (the V2E2V resolution, config c5): 563 reduction chunks per window."""
    rng = np.random.default_rng(11)
    H, W, nb = 720, 1280, 5
    ev = fx.synthetic_events(200000, H, W, rng)
    got = ep.events_to_voxel_batch([ev], nb, W, H, mode="std", filter_hot_pixel=True).cpu().numpy()
    assert_bits(got[0], fx.normalize_voxel(ref_raw(ev, nb, W, H), True, "std"))


def test_device_resident_concatenated_batch():
    """The (events, offsets) form with everything already in HBM (what bench.py times)."""
    rng = np.random.default_rng(5)
    H, W, nb = 180, 240, 5
    wins = _windows(rng, H, W, [15000] * 16)
    ev = torch.from_numpy(np.concatenate(wins)).cuda()
    off = torch.arange(0, 16 * 15000 + 1, 15000, dtype=torch.int64).cuda()
    got = ep.events_to_voxel_batch((ev, off), nb, W, H, mode="std", filter_hot_pixel=True).cpu().numpy()
    for b in (0, 7, 15):
        assert_bits(got[b], fx.normalize_voxel(ref_raw(wins[b], nb, W, H), True, "std"))
    again = ep.events_to_voxel_batch((ev, off), nb, W, H, mode="std", filter_hot_pixel=True).cpu().numpy()
    np.testing.assert_array_equal(got, again)       # deterministic


def test_gpu_voxel_loader_matches_reference_path(tmp_path):
    """f4: the GPU loader yields what train_data_loaders.py:187-193 computes per window
    (voxelize + event_preprocess(filter_hot_pixel=False)), bit-exact, in the (step, batch) layout
    of train_e2v.py:104-112."""
    from tests.test_data_readers import make_dataset
    from v2e2v_amd import data
    ds = make_dataset(tmp_path, n_lines=24)
    loader = data.GpuVoxelLoader(ds, "cuda", batch_size=2, shuffle=False, num_workers=0)
    seq_events, img, gt = next(iter(loader))
    assert len(seq_events) == 5 and seq_events[0].shape == (2, 5, 24, 32) and img.shape == (2, 1, 24, 32)
    for b in range(2):
        events, sizes, _, _ = ds[b]
        off = 0
        for s in range(5):
            win = events[off:off + int(sizes[s])].numpy()
            off += int(sizes[s])
            ref = fx.normalize_voxel(fx.voxelize(win, 5, 32, 24), filter_hot_pixel=False)
            assert_bits(seq_events[s][b], ref)


# ---- the reference's torch twins (utils/event_process.py:66-129, :157-176), pinned by
# ---- vectors the reference functions themselves produced (tests/golden/make_golden_v2e.py)
@pytest.mark.parametrize("tag,H,W", [("s", 48, 64), ("l", 180, 240)])
def test_events_to_voxel_grid_pytorch_bit_exact(golden, tag, H, W):
    d = golden("v2e_blocks.npz")
    assert_bits(ep.events_to_voxel_grid_pytorch(d[f"tv_{tag}_events"], 5, W, H), d[f"tv_{tag}_vox"])


def test_event_preprocess_pytorch_float32_statistics(golden):
    """Bar 2e-6 of max|ref|: the float32 statistics round the sums once (ATen's own float32
    reduction order is not restated); the zero mask is exact."""
    from tests.conftest import rel_err
    d = golden("v2e_blocks.npz")
    whole = ep.event_preprocess_pytorch(torch.from_numpy(d["pp_whole_in"]).cuda(), mode="std",
                                        filter_hot_pixel=False).cpu().numpy()     # v2e_model.py:526
    assert rel_err(whole, d["pp_whole_out"]) < 2e-6
    assert np.array_equal(whole == 0, d["pp_whole_out"] == 0)
    grid = ep.event_preprocess_pytorch(torch.from_numpy(d["pp_grid_in"]).cuda(), mode="std",
                                       filter_hot_pixel=True).cpu().numpy()
    assert rel_err(grid, d["pp_grid_out"]) < 2e-6
    assert np.array_equal(grid == 0, d["pp_grid_out"] == 0)
