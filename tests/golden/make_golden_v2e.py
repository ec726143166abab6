"""Golden vectors of the V2E emulator's building blocks and the reference's torch voxel twins,
computed by the REAL reference functions.  Run in the build
container only (the reference is not on the GPU box):

    PYTHONPATH=/root/reference:. python tests/golden/make_golden_v2e.py

Reference functions (they import only torch / numpy):
  v2e/emulator_utils.py:13-38   lin_log
  v2e/emulator_utils.py:41-46   rescale_intensity_frame
  v2e/emulator_utils.py:49-101  low_pass_filter (called as IIR_temporal_filtering does,
                                v2e/v2e_model.py:266-289: log_new_frame = log_frames[:, n])
  v2e/emulator_utils.py:104-126 subtract_leak_current (leak_jitter_fraction = 0: no draw matters)
  v2e/emulator_utils.py:129-162 compute_event_map
  utils/event_process.py:66-129  events_to_voxel_grid_pytorch (float64 events tensor)
  utils/event_process.py:157-176 event_preprocess_pytorch ('std', as v2e/v2e_model.py:526 calls
                                it on the whole (B, nb, H, W) tensor; and per grid with the filter)
The emulator's forward itself (v2e/v2e_model.py:290-536) cannot be imported here (the module
imports cv2); oracle/v2e_oracle.py composes these pinned blocks in its order.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import fixtures as fx  # noqa: E402
from utils import event_process as rep  # noqa: E402
from v2e import emulator_utils as eu  # noqa: E402

torch.set_num_threads(8)


def frames_fixture(F=6, H=48, W=64, seed=4):
    """Intensities 0..255 with the lin-log corner cases: 0, the threshold 20, just around it,
    255, and smooth structure (float32)."""
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    out = np.zeros((1, F, H, W), np.float32)
    for f in range(F):
        img = 40 + 30 * np.sin(xx / 5.0 + f) * np.cos(yy / 7.0) + g.uniform(0, 5, (H, W))
        img += 170 * np.exp(-((xx - 10 - 4 * f) ** 2 + (yy - H / 2) ** 2) / 60.0)
        out[0, f] = np.clip(img, 0, 255)
    out[0, :, 0, :8] = np.array([0, 20, 19.999998, 20.000002, 255, 1e-3, 5.5, 254.99998], np.float32)
    return out


def main():
    res = {}
    fr = frames_fixture()
    res["frames"] = fr
    frt = torch.from_numpy(fr)
    logf = eu.lin_log(frt)
    res["lin_log"] = logf.numpy()
    resc = eu.rescale_intensity_frame(frt)
    res["rescale"] = resc.numpy()
    # low-pass filter, one step per frame as IIR_temporal_filtering runs it
    ts = torch.linspace(0.0, 0.05, fr.shape[1], dtype=torch.float32)
    dts = ts[1:] - ts[:-1]
    res["lp_t"] = ts.numpy()
    for tag, (cut, ql, qs) in {"a": (30.0, 1.0, 1.0), "b": (15.0, 0.5, 2.0), "c": (40.0, 0.0, 1.0),
                               "d": (40.0, 1.0, 0.0)}.items():
        lp = logf[:, 0:1].clone()
        outs = []
        for n in range(1, fr.shape[1]):
            lp = eu.low_pass_filter(log_new_frame=logf[:, n], lp_log_frame0=lp, inten01=resc[:, n:n + 1],
                                    delta_time=dts[n - 1], cutoff_hz=cut, ql=ql, qs=qs)
            outs.append(lp.numpy())
        res[f"lp_{tag}"] = np.stack(outs)
        res[f"lp_{tag}_cfg"] = np.array([cut, ql, qs], np.float64)
    # leak current, deterministic (jitter 0)
    g = np.random.default_rng(8)
    base = logf[:, 0:1].clone()
    pos_thres = torch.from_numpy(np.maximum(g.normal(0.2, 0.03, base.shape), 0.01).astype(np.float32))
    noise_rate = torch.from_numpy(np.exp(np.log(10) * 0.1 * g.standard_normal(base.shape)).astype(np.float32))
    dt = torch.tensor(0.00625, dtype=torch.float32)
    res["leak_base"] = base.numpy()
    res["leak_pos_thres"] = pos_thres.numpy()
    res["leak_noise_rate"] = noise_rate.numpy()
    res["leak_out"] = eu.subtract_leak_current(base, 0.1, dt, pos_thres, 0.0, noise_rate).numpy()
    # event map of a frame difference
    diff = logf[:, 3:4] - logf[:, 0:1]
    neg_thres = torch.from_numpy(np.maximum(g.normal(0.2, 0.03, base.shape), 0.01).astype(np.float32))
    pe, ne = eu.compute_event_map(diff, pos_thres, neg_thres)
    res["em_diff"] = diff.numpy()
    res["em_neg_thres"] = neg_thres.numpy()
    res["em_pos"] = pe.numpy()
    res["em_neg"] = ne.numpy()
    # torch voxel twins
    for tag, (H, W, n, seed) in {"s": (48, 64, 1200, 21), "l": (180, 240, 15000, 22)}.items():
        ev = fx.synthetic_events(n, H, W, np.random.default_rng(seed))
        res[f"tv_{tag}_events"] = ev
        res[f"tv_{tag}_vox"] = rep.events_to_voxel_grid_pytorch(torch.from_numpy(ev.copy()), 5, W, H).numpy()
    # event_preprocess_pytorch as the emulator calls it: whole (B, nb, H, W) tensor, no filter
    raw = np.stack([res["tv_s_vox"], 2.0 * res["tv_s_vox"][::-1]]).astype(np.float32)
    res["pp_whole_in"] = raw
    res["pp_whole_out"] = rep.event_preprocess_pytorch(torch.from_numpy(raw.copy()), mode="std",
                                                       filter_hot_pixel=False).numpy()
    # and per grid with the hot-pixel filter (threshold 20 / num_bins), on a grid with hot pixels
    hot = res["tv_l_vox"].copy()
    hot[:, 10, 10] = 7.5
    hot[2, 100, 200] = -9.0
    res["pp_grid_in"] = hot
    res["pp_grid_out"] = rep.event_preprocess_pytorch(torch.from_numpy(hot.copy()), mode="std",
                                                      filter_hot_pixel=True).numpy()
    path = os.path.join(HERE, "v2e_blocks.npz")
    np.savez_compressed(path, **res)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
