"""Generate tests/golden/vox_spill.npz by running the REAL reference voxelisers on event windows
whose events partly lie outside the H x W frame but inside the grid ("spill": x >= W, y >= H or a
negative x, added by np.add.at / index_add_ to another pixel or bin of the grid).

Run in the build container only (the reference tree does not exist on the GPU box):

    PYTHONPATH=/root/reference:. python tests/golden/make_golden_spill.py

It imports ``utils.event_process`` (reference ``utils/event_process.py:15-63`` numpy path and
``:66-129`` torch path) unmodified and writes data only: per window the events and both
reference grids (``np_<k>`` and ``torch_<k>``; ``torch_ok_<k>`` = 0 where the torch path raises,
i.e. a negative flat index, which np.add.at counts from the end of the grid instead).

Windows (nb = 5 bins):
  0  20 x 30, 3000 in-frame events + 90 spilled (x >= W, x <= -1 with y >= 1, y >= H at early t,
     fractional x in [W, W+1)) -- many in-frame events on the spill targets, so the order in
     which the adds reach a cell is exercised;
  1  20 x 30, as 0 plus x = -3 at y = 0 in the first bin: the index is negative (the end of the
     grid in numpy; the torch path raises);
  2  64 x 64, 40000 events (three 16384-event segments of the fused GPU path) + 300 spilled;
  3  520 x 520 (>= 2^18 pixels: the global-sort GPU path), 30000 events + 200 spilled.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import fixtures as fx  # noqa: E402

from utils import event_process as ref_ev  # noqa: E402  (reference, PYTHONPATH=/root/reference)

NB = 5


def spill_window(rng, H, W, n, n_spill, neg_wrap=False):
    ev = fx.synthetic_events(n, H, W, rng)
    t = ev[:, 0]
    t0, t1 = t[0], t[-1]
    sp = []
    for i in range(n_spill):
        kind = i % 4
        tt = rng.uniform(t0, t1)
        if kind == 0:                               # x >= W: the next row's pixel, same bin
            x, y = W + rng.integers(0, 6), rng.integers(0, H - 1)
        elif kind == 1:                             # x <= -1 (y >= 1): the previous row's end
            x, y = -float(rng.integers(1, 5)) - rng.uniform(0, 0.9), rng.integers(1, H)
        elif kind == 2:                             # y >= H at an early time: a later bin
            x, y = rng.integers(0, W), H + rng.integers(0, H)
            tt = rng.uniform(t0, t0 + (t1 - t0) * 0.45)    # ti <= 1: bins ti + 1 .. ti + 3 < NB
        else:                                       # fractional x in [W, W + 1): truncates to W
            x, y = W + rng.uniform(0.0, 0.99), rng.integers(0, H - 1)
        sp.append([tt, x, y, rng.integers(0, 2)])
    if neg_wrap:                                    # flat index -3 + bin 0: numpy wraps, torch raises
        sp.append([t0 + (t1 - t0) * 0.01, -3.0, 0.0, 1.0])
    # in-frame events on some spill targets (same cells, interleaved in time)
    for row in list(sp[: n_spill // 3]):
        x, y = row[1], row[2]
        if x >= W:
            px, py = int(x) - W, int(y) + 1
        elif x <= -1:
            px, py = W + int(x), int(y) - 1
        else:
            continue
        for _ in range(3):
            sp.append([rng.uniform(t0, t1), px, py, rng.integers(0, 2)])
    ev = np.concatenate([ev, np.asarray(sp, np.float64)])
    # keep the window's first and last events in place (they fix the time normalisation)
    mid = ev[1:]
    mid = mid[np.argsort(mid[:, 0], kind="stable")]
    ev = np.concatenate([ev[:1], mid])
    ev[-1, 0] = max(ev[-1, 0], t1)
    return ev


def main():
    rng = np.random.default_rng(2026)
    specs = [(20, 30, 3000, 90, False), (20, 30, 3000, 90, True), (64, 64, 40000, 300, False),
             (520, 520, 30000, 200, False)]
    out = {}
    for k, (H, W, n, ns, neg) in enumerate(specs):
        ev = spill_window(rng, H, W, n, ns, neg)
        out[f"events_{k}"] = ev
        out[f"shape_{k}"] = np.array([NB, H, W])
        out[f"np_{k}"] = ref_ev.events_to_voxel_grid(ev.copy(), NB, W, H).astype(np.float32)
        try:
            g = ref_ev.events_to_voxel_grid_pytorch(torch.from_numpy(ev.copy()), NB, W, H)
            out[f"torch_{k}"] = g.numpy().astype(np.float32)
            out[f"torch_ok_{k}"] = np.array(1)
        except (IndexError, RuntimeError):
            out[f"torch_{k}"] = np.zeros((NB, H, W), np.float32)
            out[f"torch_ok_{k}"] = np.array(0)
        outside = (ev[:, 1] <= -1) | (ev[:, 1] >= W) | (ev[:, 2] <= -1) | (ev[:, 2] >= H)
        print(f"window {k}: {H}x{W}, {len(ev)} events, {int(outside.sum())} outside the frame, "
              f"torch ok {int(out[f'torch_ok_{k}'])}")
    np.savez_compressed(os.path.join(HERE, "vox_spill.npz"), **out)


if __name__ == "__main__":
    main()
