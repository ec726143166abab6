"""Pins oracle/v2e_oracle.py's building blocks to vectors the REAL reference functions produced
(tests/golden/make_golden_v2e.py): v2e/emulator_utils.py
lin_log / rescale_intensity_frame / low_pass_filter / subtract_leak_current / compute_event_map
and utils/event_process.py events_to_voxel_grid_pytorch / event_preprocess_pytorch.

Bars: bit-exact wherever the reference's arithmetic is elementwise float32/float64 and
sequential; event_preprocess_pytorch within 2e-6 of max|ref| (ATen's float32 sum order is not
restated: the oracle rounds the exact sum once, so mean / std may differ by an ulp)."""
import numpy as np
import pytest

from oracle import v2e_oracle as vo
from tests.conftest import rel_err


@pytest.fixture(scope="module")
def d(golden):
    return golden("v2e_blocks.npz")


def test_lin_log_and_rescale_bit_exact(d):
    assert np.array_equal(vo.lin_log(d["frames"]), d["lin_log"])
    assert np.array_equal(vo.rescale_intensity_frame(d["frames"]), d["rescale"])


@pytest.mark.parametrize("tag", ["a", "b", "c", "d"])
def test_low_pass_filter_bit_exact(d, tag):
    cut, ql, qs = d[f"lp_{tag}_cfg"]
    logf, resc, t = d["lin_log"], d["rescale"], d["lp_t"]
    lp = logf[:, 0:1]
    for n in range(1, logf.shape[1]):
        lp = vo.low_pass_filter(logf[:, n:n + 1], lp, resc[:, n:n + 1], np.float32(t[n] - t[n - 1]), cut, ql, qs)
        assert np.array_equal(lp, d[f"lp_{tag}"][n - 1]), n


def test_subtract_leak_current_bit_exact(d):
    out = vo.subtract_leak_current(d["leak_base"], 0.1, np.float32(0.00625), d["leak_pos_thres"], 0.0,
                                   d["leak_noise_rate"], np.zeros_like(d["leak_base"]))
    assert np.array_equal(out, d["leak_out"])


def test_compute_event_map_bit_exact(d):
    pe, ne = vo.compute_event_map(d["em_diff"], d["leak_pos_thres"], d["em_neg_thres"])
    assert np.array_equal(pe, d["em_pos"]) and np.array_equal(ne, d["em_neg"])
    assert d["em_pos"].max() > 0 and d["em_neg"].max() > 0


@pytest.mark.parametrize("tag,H,W", [("s", 48, 64), ("l", 180, 240)])
def test_events_to_voxel_grid_pytorch_bit_exact(d, tag, H, W):
    assert np.array_equal(vo.events_to_voxel_grid_pytorch(d[f"tv_{tag}_events"], 5, W, H), d[f"tv_{tag}_vox"])


def test_event_preprocess_pytorch(d):
    assert rel_err(vo.preprocess_whole(d["pp_whole_in"]), d["pp_whole_out"]) < 2e-6
    assert rel_err(vo.event_preprocess_pytorch(d["pp_grid_in"], "std", True), d["pp_grid_out"]) < 2e-6
    # the zero pattern (mask) is exact
    assert np.array_equal(vo.preprocess_whole(d["pp_whole_in"]) == 0, d["pp_whole_out"] == 0)
