"""GPU event voxelizer: the MI355X twin of reference ``utils/event_process.py``.

Drop-in names:

* ``events_to_voxel_grid(events, num_bins, width, height)``      <- utils/event_process.py:15-63
* ``events_to_voxel_grid_pytorch(events, num_bins, width, height)`` <- utils/event_process.py:66-129
* ``event_preprocess(voxel, mode='std', filter_hot_pixel=False)`` <- utils/event_process.py:132-154
* ``event_preprocess_pytorch(voxel, mode, filter_hot_pixel=True)``<- utils/event_process.py:157-176
* ``events_to_voxel_batch(windows, ...)``: many windows -> (B, num_bins, H, W) in one launch
  sequence (what the data readers need per sequence: data_readers/train_data_loaders.py:187-193,
  data_readers/video_readers.py:161-178).

All of them run in libcista_hip.so (include/cista_voxel.h) and return CUDA tensors.  The numpy
twins are bit-identical to the reference's numpy path (voxel accumulation order, numpy's float32
pairwise reduction for the 'std' statistics); the torch twins follow the reference's torch
arithmetic: events_to_voxel_grid_pytorch bit-identically (float32 contributions, float32
index_add_), event_preprocess_pytorch with float32 statistics (its sum() rounded once: ATen's
reduction order may differ in the last bit, tests/test_gpu_voxel.py bounds it at 2e-6).  Events
outside the H x W frame are treated as the reference's flat index treats them: added to the
pixel / bin it lands on (bit-identically, in event order with that cell's own events), or
IndexError where the reference raises.  Difference from the reference, by design: inputs are
never modified (the reference rewrites ``events[:, 0]``, the polarity column, and the voxel grid
when filtering hot pixels).  There is no CPU fallback: without the HIP library every call raises.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

MODES = {"none": 0, "raw": 0, "std": 1, "maxmin": 2}
STD_F32 = 3                 # CISTA_VOXEL_STD_F32: event_preprocess_pytorch's float32 statistics
TORCH_ACCUM = 0x10          # CISTA_VOXEL_TORCH_ACCUM: events_to_voxel_grid_pytorch accumulation
OUT_OF_RANGE, SPILL = 1, 2  # cista_voxelize_checked grid_status bits (include/cista_voxel.h)
_ws_cache: dict = {}


def _device(dev=None) -> torch.device:
    if dev is not None:
        return torch.device(dev)
    if not torch.cuda.is_available():
        raise _lib.CistaError("the event voxelizer runs on a ROCm GPU only (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def _workspace(device, nbytes: int) -> torch.Tensor:
    key = (device.type, device.index)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf


def _as_events(ev, device) -> torch.Tensor:
    if isinstance(ev, np.ndarray):
        ev = torch.from_numpy(np.ascontiguousarray(ev))
    if ev.dim() != 2 or ev.shape[1] != 4:
        raise AssertionError("events must be an [N x 4] array (t, x, y, p)")   # reference :22
    return ev.to(device=device, dtype=torch.float64).contiguous()


def _threshold(filter_hot_pixel: bool, num_bins: int, per_bin: float) -> float:
    return float(np.float32(per_bin / num_bins)) if filter_hot_pixel else 0.0


def events_to_voxel_batch(windows, num_bins: int, width: int, height: int, mode: str = "none",
                          filter_hot_pixel: bool = False, hot_threshold: float | None = None,
                          out: torch.Tensor | None = None, device=None, torch_semantics: bool = False,
                          strict: bool = True) -> torch.Tensor:
    """Voxelize (and optionally normalise) B event windows at once.

    ``windows`` is either a list of [N_b x 4] arrays/tensors (t, x, y, p), or a pair
    ``(events, offsets)`` with all windows concatenated (device tensors stay on the device).
    ``mode`` is 'none' (events_to_voxel_grid only), 'std' or 'maxmin' (event_preprocess);
    ``filter_hot_pixel`` uses the numpy threshold 25/num_bins unless ``hot_threshold`` is given.
    ``torch_semantics``: the torch twins' arithmetic (events_to_voxel_grid_pytorch accumulation,
    event_preprocess_pytorch float32 'std' statistics) instead of the numpy path's.
    Events outside the H x W frame go where the reference's flat index x + y*W + bin*H*W puts them
    (utils/event_process.py:53-58 ``np.add.at``, :113-124 ``index_add_``): an event the reference
    adds to another pixel or bin (x >= W, y >= H or a negative x, at an index inside the grid) is
    added there, bit-identically.  ``strict`` (default): an index the reference rejects raises
    IndexError as there (one stream synchronisation); ``strict=False`` skips the check and drops
    such events.
    Returns (B, num_bins, height, width) float32 on the GPU.
    """
    if num_bins <= 0 or width <= 0 or height <= 0:
        raise AssertionError("num_bins, width and height must be positive")   # reference :23-25
    dev = _device(device)
    if isinstance(windows, tuple):
        events, offsets = windows
        events = _as_events(events, dev)
        offsets = torch.as_tensor(offsets, dtype=torch.int64).to(dev).contiguous()
    else:
        parts = [_as_events(w, dev) for w in windows]
        sizes = [p.shape[0] for p in parts]
        events = torch.cat(parts, 0) if parts else torch.zeros(0, 4, dtype=torch.float64, device=dev)
        offsets = torch.tensor(np.concatenate([[0], np.cumsum(sizes)]), dtype=torch.int64, device=dev)
    B = offsets.numel() - 1
    N = events.shape[0]
    if out is None:
        out = torch.empty(B, num_bins, height, width, dtype=torch.float32, device=dev)
    elif out.shape != (B, num_bins, height, width) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous float32 (B, num_bins, height, width) tensor")
    thr = hot_threshold if hot_threshold is not None else _threshold(filter_hot_pixel, num_bins, 25.0)
    m = MODES[mode]
    if torch_semantics:
        m = (STD_F32 if m == MODES["std"] else m) | TORCH_ACCUM
    L = _lib.lib()
    nbytes = L.cista_voxel_workspace_bytes(B, N, num_bins, height, width)
    ws = _workspace(dev, nbytes)
    status = torch.zeros(1, dtype=torch.int32, device=dev) if strict else None
    with torch.cuda.device(dev):
        _lib.check(L.cista_voxelize_checked(_lib.ptr(events) if N else None, offsets.data_ptr(), B, N, num_bins,
                                            height, width, m, ctypes.c_float(thr), out.data_ptr(), ws.data_ptr(),
                                            ws.numel(), _lib.ptr(status), _lib.stream_handle(dev)),
                   "cista_voxelize_checked")
    if strict:
        flags = int(status.item())
        if flags & OUT_OF_RANGE:
            raise IndexError(f"index out of bounds for a voxel grid of size {num_bins * height * width}: an event's "
                             f"x, y lie outside the {height}x{width} frame (np.add.at raises here, "
                             "utils/event_process.py:53-58)")
    return out


def events_to_voxel_grid(events, num_bins: int, width: int, height: int) -> torch.Tensor:
    """Reference utils/event_process.py:15-63 on the GPU: (num_bins, height, width) float32."""
    return events_to_voxel_batch([events], num_bins, width, height)[0]


def events_to_voxel_grid_pytorch(events, num_bins: int, width: int, height: int) -> torch.Tensor:
    """Reference utils/event_process.py:66-129 on the GPU (a float64 events tensor's arithmetic):
    (num_bins, height, width) float32."""
    return events_to_voxel_batch([events], num_bins, width, height, torch_semantics=True)[0]


def _preprocess(vox: torch.Tensor, mode: str, thr: float, f32_stats: bool = False) -> torch.Tensor:
    if not vox.is_cuda:
        raise _lib.CistaError("event_preprocess runs on a ROCm GPU only; move the voxel grid to cuda")
    squeeze = vox.dim() == 3
    v = vox.unsqueeze(0) if squeeze else vox
    if v.dim() != 4:
        raise ValueError("voxel grid must be (num_bins, H, W) or (B, num_bins, H, W)")
    res = v.to(torch.float32).contiguous().clone()
    B, nb, H, W = res.shape
    L = _lib.lib()
    ws = _workspace(res.device, L.cista_voxel_workspace_bytes(B, 0, nb, H, W))
    with torch.cuda.device(res.device):
        m = STD_F32 if (f32_stats and mode == "std") else MODES[mode]
        _lib.check(L.cista_voxel_preprocess(res.data_ptr(), B, nb, H, W, m, ctypes.c_float(thr),
                                            ws.data_ptr(), ws.numel(), _lib.stream_handle(res.device)),
                   "cista_voxel_preprocess")
    return res[0] if squeeze else res


def event_preprocess(event_voxel_grid: torch.Tensor, mode: str = "std", filter_hot_pixel: bool = False):
    """Reference utils/event_process.py:132-154 (hot-pixel threshold 25/num_bins)."""
    nb = event_voxel_grid.shape[-3]
    return _preprocess(event_voxel_grid, mode, _threshold(filter_hot_pixel, nb, 25.0))


def event_preprocess_pytorch(event_voxel_grid: torch.Tensor, mode: str = "std", filter_hot_pixel: bool = True):
    """Reference utils/event_process.py:157-176 (hot-pixel threshold 20/num_bins, float32
    statistics).  Like the reference, the statistics span the WHOLE tensor it is given: a
    (num_bins, H, W) grid, or a (B, num_bins, H, W) batch as v2e/v2e_model.py:526 passes it
    (the threshold then uses the reference's shape[0])."""
    nb = event_voxel_grid.shape[0]
    v = event_voxel_grid
    if v.dim() == 4:                    # one statistics window over the whole batch
        B, n1, H, W = v.shape
        return _preprocess(v.reshape(1, B * n1, H, W), mode, _threshold(filter_hot_pixel, nb, 20.0),
                           f32_stats=True).reshape(B, n1, H, W)
    return _preprocess(v, mode, _threshold(filter_hot_pixel, nb, 20.0), f32_stats=True)
