"""Deterministic input / weight recipes shared by the golden-fixture script and the tests.

TEST INFRASTRUCTURE ONLY -- nothing under ``oracle/`` is imported by the product package
(``v2e2v_amd``).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use it.

Recipes follow SURVEY.md section 8(c):

* synthetic events: per frame ``n`` events with t = sort(U(0, 0.05)), x ~ U{0..W-1},
  y ~ U{0..H-1}, p ~ U{0, 1};
* voxelisation restates ``events_to_voxel_grid`` (reference ``utils/event_process.py:15-63``)
  and ``event_preprocess(mode='std', filter_hot_pixel=True)`` (``utils/event_process.py:132-154``),
  result cast to float32 (under numpy 2 the reference returns float64);
* "stress" weights: conv weight ~ N(0, 1/fan_in), bias ~ U(-0.1, 0.1), Lambda = 0.05 --
  the default PyTorch init gives an almost constant 0.5 output and proves little.
"""
from __future__ import annotations

import numpy as np

# parameter order of CistaLSTCNet.state_dict() (reference e2v/e2v_model.py:6-38,
# e2v/base_layers.py) -- unique tensors only; lista_blocks.{0..depth-1} are one tied module.
def param_shapes(base_channels: int = 64, depth: int = 5, num_bins: int = 5):
    C = base_channels
    h = C // 2
    return [
        ("We.conv2d.weight", (h, num_bins, 3, 3)), ("We.conv2d.bias", (h,)),
        ("Wi.conv2d.weight", (h, 1, 3, 3)), ("Wi.conv2d.bias", (h,)),
        ("W0.conv2d.weight", (C, C, 3, 3)), ("W0.conv2d.bias", (C,)),
        ("P0.gates.weight", (4 * C, 3 * C, 3, 3)), ("P0.gates.bias", (4 * C,)),
        ("P0.out_gates.weight", (2 * C, 4 * C, 3, 3)), ("P0.out_gates.bias", (2 * C,)),
        ("P0.P0.weight", (2 * C, C, 3, 3)), ("P0.P0.bias", (2 * C,)),
        ("lista.Lambda", (1, 2 * C, 1, 1)),
        ("lista.D.conv2d.weight", (C, 2 * C, 3, 3)), ("lista.D.conv2d.bias", (C,)),
        ("lista.P.conv2d.weight", (2 * C, C, 3, 3)), ("lista.P.conv2d.bias", (2 * C,)),
        ("Dg.conv.conv2d.weight", (C, 2 * C, 3, 3)), ("Dg.conv.conv2d.bias", (C,)),
        ("Dg.recurrent_block.Gates.weight", (4 * C, 2 * C, 3, 3)),
        ("Dg.recurrent_block.Gates.bias", (4 * C,)),
        ("upsamp_conv.conv2d.weight", (C, C, 3, 3)), ("upsamp_conv.conv2d.bias", (C,)),
        ("final_conv.conv2d.weight", (1, C, 3, 3)), ("final_conv.conv2d.bias", (1,)),
    ]


def expand_tied(params: dict, depth: int) -> dict:
    """Unique-parameter dict -> the reference's 45-key state_dict layout (tied ISTA copies)."""
    out = {}
    for k, v in params.items():
        if k.startswith("lista."):
            continue
        out[k] = v
    # reference key order: ... P0.*, lista_blocks.i.{Lambda, D.*, P.*}, Dg.*, ...
    ordered = {}
    for k, v in out.items():
        if k.startswith("Dg.") and not any(x.startswith("lista_blocks.") for x in ordered):
            for i in range(depth):
                ordered[f"lista_blocks.{i}.Lambda"] = params["lista.Lambda"]
                ordered[f"lista_blocks.{i}.D.conv2d.weight"] = params["lista.D.conv2d.weight"]
                ordered[f"lista_blocks.{i}.D.conv2d.bias"] = params["lista.D.conv2d.bias"]
                ordered[f"lista_blocks.{i}.P.conv2d.weight"] = params["lista.P.conv2d.weight"]
                ordered[f"lista_blocks.{i}.P.conv2d.bias"] = params["lista.P.conv2d.bias"]
        ordered[k] = v
    return ordered


def collapse_tied(state_dict: dict, depth: int) -> dict:
    """45-key state_dict -> unique params.  The LAST tied copy wins, as the reference's
    load_state_dict does ('Tied weights')."""
    out = {}
    for k, v in state_dict.items():
        if k.startswith("lista_blocks."):
            rest = k.split(".", 2)[2]
            out["lista." + rest] = v
        else:
            out[k] = v
    return out


def stress_params(base_channels=64, depth=5, num_bins=5, seed=7, lam=0.05):
    """He-scaled random weights (unique tensors, float32 numpy)."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in param_shapes(base_channels, depth, num_bins):
        if name.endswith("Lambda"):
            out[name] = np.full(shape, lam, np.float32)
        elif name.endswith("weight"):
            fan_in = int(np.prod(shape[1:]))
            out[name] = (rng.standard_normal(shape) / np.sqrt(fan_in)).astype(np.float32)
        else:
            out[name] = rng.uniform(-0.1, 0.1, shape).astype(np.float32)
    return out


def synthetic_events(n: int, H: int, W: int, rng: np.random.Generator) -> np.ndarray:
    """[n, 4] float64 events (t, x, y, p), t sorted in [0, 0.05)."""
    t = np.sort(rng.uniform(0.0, 0.05, n))
    x = rng.integers(0, W, n)
    y = rng.integers(0, H, n)
    p = rng.integers(0, 2, n)
    return np.stack([t, x, y, p], 1).astype(np.float64)


def voxelize(events: np.ndarray, num_bins: int, W: int, H: int) -> np.ndarray:
    """Temporal-bilinear voxel grid; restates reference utils/event_process.py:15-63
    (does NOT mutate its input, unlike the reference :40,45)."""
    vox = np.zeros(num_bins * H * W, np.float32)
    if len(events) == 0:
        return vox.reshape(num_bins, H, W)
    t = events[:, 0].astype(np.float64)
    dT = t[-1] - t[0]
    if dT == 0:
        dT = 1.0
    ts = (num_bins - 1) * (t - t[0]) / dT                      # :40
    xs = events[:, 1].astype(np.uint64)
    ys = events[:, 2].astype(np.uint64)
    pol = events[:, 3].astype(np.float64).copy()
    pol[pol == 0] = -1                                          # :45
    ti = ts.astype(np.uint64)
    dt = ts - ti
    vl = pol * (1.0 - dt)
    vr = pol * dt
    ok = ti < num_bins
    np.add.at(vox, xs[ok] + ys[ok] * W + ti[ok] * W * H, vl[ok])          # :53-54
    ok = (ti + 1) < num_bins
    np.add.at(vox, xs[ok] + ys[ok] * W + (ti[ok] + 1) * W * H, vr[ok])    # :57-58
    return vox.reshape(num_bins, H, W)


def normalize_voxel(vox: np.ndarray, filter_hot_pixel: bool = True, mode: str = "std",
                    per_bin: float = 25.0) -> np.ndarray:
    """Restates event_preprocess (reference utils/event_process.py:132-154; per_bin=20 gives the
    hot-pixel threshold of event_preprocess_pytorch :157-162); computes in float64 like the
    reference does under numpy 2, returns float32."""
    v = vox.astype(np.float32).copy()
    nb = v.shape[0]
    if filter_hot_pixel:
        v[np.abs(v) > per_bin / nb] = 0                             # :137-138
    if mode == "maxmin":                                            # :139-140
        return np.asarray((v - v.min()) / (v.max() - v.min() + 1e-8), dtype=np.float32)
    if mode != "std":
        return v
    nz = v != 0
    n = nz.sum()
    if n > 0:
        mean = v.sum() / n                                          # float32 sum, :148
        mask = nz.astype(np.float32)
        std = np.sqrt((v ** 2).sum() / n - mean ** 2)               # :150
        v = mask * (v - mean) / (std + 1e-8)
    return np.asarray(v, dtype=np.float32)


def synthetic_voxels(n_frames: int, B: int, num_bins: int, H: int, W: int,
                     n_events: int = 15000, seed: int = 1234) -> np.ndarray:
    """[n_frames, B, num_bins, H, W] float32 voxels."""
    out = np.zeros((n_frames, B, num_bins, H, W), np.float32)
    for b in range(B):
        rng = np.random.default_rng(seed + b)
        for f in range(n_frames):
            ev = synthetic_events(n_events, H, W, rng)
            out[f, b] = normalize_voxel(voxelize(ev, num_bins, W, H))
    return out


def density_matched_events(H: int, W: int, n_full: int = 15000) -> int:
    """Event count for a smaller frame at the 180x240 density."""
    return max(1, int(round(n_full * H * W / (180 * 240))))
