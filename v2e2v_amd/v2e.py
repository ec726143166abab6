"""Video-to-events emulator and the V2E2V pipeline on the GPU.

``EventEmulator`` mirrors reference v2e/v2e_model.py:31-536 (same constructor arguments and
defaults, ``reset()``, ``forward(frames, t_frames) -> (events, num_events)``) in both output
modes: ``'voxel_grid'``, the mode V2E2VNet uses (model_v2e2v.py:28-29,46-61), and ``'raw'``, the
sorted [t, x, y, p, b] event list (:504-518,527-534); the whole frame step runs in
libcista_hip.so (include/cista_v2e.h).  ``V2E2VNet`` mirrors model_v2e2v.py:9-128: emulator + the
drop-in CistaLSTCNet.

Differences, by design: random draws come from a counter-based Philox stream keyed by ``seed``
(statistically the reference's torch.normal / randn / rand, not the same numbers); ``seed=0``
draws a fresh seed like the reference's unseeded torch RNG.  Raw rows of equal (b, t) keep their
emission order (y, x), which the reference's unstable torch.sort does not promise.  The cv2
state display is not built (V2E2V never uses it).
"""
from __future__ import annotations

import ctypes
import numbers
import random

import numpy as np
import torch

from . import _lib
from .e2v_model import CistaLSTCNet


class CistaV2EConfig(ctypes.Structure):
    _fields_ = [("num_bins", ctypes.c_int)] + [(n, ctypes.c_float) for n in (
        "pl", "ps", "ql", "qs", "pos_thres", "neg_thres", "sigma_thres", "cutoff_hz", "leak_rate_hz",
        "refractory_period_s", "shot_noise_rate_hz", "leak_jitter_fraction", "noise_rate_cov_decades")] + [
        ("seed", ctypes.c_ulonglong)]


class CistaV2EHostState(ctypes.Structure):
    _fields_ = [("initialized", ctypes.c_int), ("t_previous", ctypes.c_float), ("draw", ctypes.c_ulonglong)]


class EventCount(numbers.Integral):
    """The emulator's event count kept on the device until it is read -- the opt-in
    ``lazy_count=True`` mode of EventEmulator, for pipelines that must not host-sync once per pack
    (the default returns a plain Python int, as the reference does, v2e_model.py:536).  A full
    numbers.Integral: int(), operator.index, comparisons, hashing, arithmetic, //, %, **, bit
    operations and formatting all act on the integer value (read once, on first use).  It is not
    an ``int`` instance (an int's value is fixed when it is made, and this one is not known until
    the GPU has run): ``isinstance(n, int)`` and json need ``int(n)``."""

    __slots__ = ("_t", "_v")

    def __init__(self, t):
        self._t, self._v = t, None

    def __int__(self):
        if self._v is None:
            self._v = int(self._t.item())
            self._t = None
        return self._v

    def __index__(self):
        return int(self)

    def __float__(self):
        return float(int(self))

    def __complex__(self):
        return complex(int(self))

    def __bool__(self):
        return int(self) != 0

    def __hash__(self):
        return hash(int(self))

    def __repr__(self):
        return repr(int(self))

    __str__ = __repr__

    def __format__(self, spec):
        return format(int(self), spec)

    def __round__(self, ndigits=None):
        return int(self) if ndigits is None else round(int(self), ndigits)

    def __trunc__(self):
        return int(self)

    def __floor__(self):
        return int(self)

    def __ceil__(self):
        return int(self)

    @property
    def numerator(self):
        return int(self)

    @property
    def denominator(self):
        return 1

    def __eq__(self, o):
        return int(self) == o

    def __lt__(self, o):
        return int(self) < o

    def __le__(self, o):
        return int(self) <= o

    def __gt__(self, o):
        return int(self) > o

    def __ge__(self, o):
        return int(self) >= o

    def __neg__(self):
        return -int(self)

    def __pos__(self):
        return int(self)

    def __abs__(self):
        return abs(int(self))

    def __invert__(self):
        return ~int(self)

    def __pow__(self, o, mod=None):
        return pow(int(self), o, mod)

    def __rpow__(self, o, mod=None):
        return pow(o, int(self), mod)


def _binop(name):
    def fwd(self, o):
        return getattr(int(self), name)(o)

    def rev(self, o):
        return getattr(int(self), "__r" + name[2:])(o)
    return fwd, rev


for _op in ("__add__", "__sub__", "__mul__", "__truediv__", "__floordiv__", "__mod__", "__divmod__",
            "__lshift__", "__rshift__", "__and__", "__xor__", "__or__"):
    _f, _r = _binop(_op)
    setattr(EventCount, _op, _f)
    setattr(EventCount, "__r" + _op[2:], _r)
EventCount.__abstractmethods__ = frozenset()


class EventEmulator(torch.nn.Module):
    """v2e_model.py:31-156 constructor surface."""

    def __init__(self, output_mode, pl=1, ps=1, ql=1, qs=1, num_bins=5, pos_thres=0.2, neg_thres=0.2,
                 sigma_thres=0.03, cutoff_hz=0, leak_rate_hz=0.1, refractory_period_s=0, shot_noise_rate_hz=0,
                 leak_jitter_fraction=0.1, noise_rate_cov_decades=0.1, seed=0, show_dvs_model_state=None,
                 device="cuda", lazy_count=False):
        super().__init__()
        if output_mode not in ("voxel_grid", "raw"):
            raise ValueError(f"output_mode must be 'voxel_grid' or 'raw', not {output_mode!r}")
        if show_dvs_model_state:
            raise NotImplementedError("the cv2 model-state display is not built")
        self.output_mode = output_mode
        self.num_bins = num_bins
        self.device = torch.device(device)
        self.cfg = CistaV2EConfig(num_bins, pl, ps, ql, qs, pos_thres, neg_thres, sigma_thres, cutoff_hz,
                                  leak_rate_hz, refractory_period_s, shot_noise_rate_hz, leak_jitter_fraction,
                                  noise_rate_cov_decades, seed if seed != 0 else random.getrandbits(63))
        self.hs = CistaV2EHostState(0, 0.0, 0)
        self.state = None
        self.num_events = 0
        self.frame_counter = 0
        self._shape = None
        self.lazy_count = lazy_count   # True: num_events is an EventCount (no host sync per call)
        self._rows = None              # raw mode: the event-row buffer, grown on demand
        self.ws = None

    def reset(self):
        """v2e_model.py:255-263: the next forward re-initialises the base frame."""
        self.hs.initialized = 0
        self.frame_counter = 0

    def forward(self, frames, t_frames):
        """frames (B, F, H, W) intensities 0..255; t_frames (B, 2) or (B, F) seconds.
        Returns (voxels (B, num_bins, H, W), num_events) in voxel_grid mode, (events (N, 5) float32
        rows [t, x, y, p, b], num_events) in raw mode (v2e_model.py:290-536)."""
        if not frames.is_cuda:
            raise _lib.CistaError("the event emulator runs on a ROCm GPU only (no CPU fallback)")
        B, F, H, W = frames.shape
        self.frame_counter += F
        fr = frames.detach().to(torch.float32).contiguous()
        tf = np.ascontiguousarray(torch.as_tensor(t_frames).detach().cpu().to(torch.float64).numpy())
        if tf.ndim != 2 or tf.shape[0] != B or tf.shape[1] not in (2, F):
            raise ValueError("t_frames must be (batch, 2) or (batch, num_frames)")
        L = _lib.lib()
        raw = self.output_mode == "raw"
        if self.state is None or self._shape != (B, H, W) or self.state.device != fr.device:
            self.state = torch.empty(L.cista_v2e_state_bytes(B, H, W), dtype=torch.uint8, device=fr.device)
            self._shape = (B, H, W)
            self.ws = None
            self.hs.initialized = 0
        if self.ws is None:
            nbytes = (L.cista_v2e_raw_workspace_bytes if raw else L.cista_v2e_workspace_bytes)(B, H, W)
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=fr.device)
        stream = _lib.stream_handle(fr.device)
        if raw:
            return self._forward_raw(L, fr, tf, B, F, H, W, stream)
        out = torch.empty(B, self.num_bins, H, W, device=fr.device)
        nev = torch.zeros(1, dtype=torch.int64, device=fr.device)
        status = L.cista_v2e_forward(ctypes.byref(self.cfg), ctypes.byref(self.hs), self.state.data_ptr(),
                                     fr.data_ptr(), tf.ctypes.data, tf.shape[1], B, F, H, W, out.data_ptr(),
                                     nev.data_ptr(), self.ws.data_ptr(), self.ws.numel(), stream)
        self._check_status(status, "cista_v2e_forward")
        # the reference returns a Python int; lazy_count keeps it on the device until it is read
        self.num_events = EventCount(nev) if self.lazy_count else int(nev.item())
        return out, self.num_events

    def _check_status(self, status, what):
        if status == 1 and self.hs.initialized:
            raise ValueError("this frame time must be later than previous frame time")   # :339-342
        _lib.check(status, what)

    def _forward_raw(self, L, fr, tf, B, F, H, W, stream):
        """Raw rows [t, x, y, p, b] sorted by b then t (:527-534); t in voxel-time units as the
        reference emits them.  The library reports the event count first when the row buffer is
        too small (the emulator state untouched), so the buffer grows and the call repeats once."""
        n = ctypes.c_ulonglong(0)
        loops = ctypes.c_int(0)
        for attempt in range(2):
            cap = 0 if self._rows is None else self._rows.shape[0]
            status = L.cista_v2e_forward_raw(ctypes.byref(self.cfg), ctypes.byref(self.hs), self.state.data_ptr(),
                                             fr.data_ptr(), tf.ctypes.data, tf.shape[1], B, F, H, W,
                                             None if self._rows is None else self._rows.data_ptr(), cap,
                                             ctypes.byref(n), ctypes.byref(loops), self.ws.data_ptr(),
                                             self.ws.numel(), stream)
            if status == 4 and attempt == 0:          # CISTA_ERR_WORKSPACE: rows needed = n
                self._rows = torch.empty(max(int(n.value), 2 * cap), 5, dtype=torch.float32, device=fr.device)
                continue
            self._check_status(status, "cista_v2e_forward_raw")
            break
        self.num_events = int(n.value)
        if loops.value == 0:                          # no iteration ran: torch.tensor([]) (:347)
            return torch.zeros(0, device=fr.device), self.num_events
        if self._rows is None:                        # iterations ran, but every event was filtered out
            return torch.zeros(0, 5, device=fr.device), self.num_events
        return self._rows[:self.num_events].clone(), self.num_events


class V2E2VNet(torch.nn.Module):
    """model_v2e2v.py:9-128: EventEmulator (voxel grid) -> CistaLSTCNet."""

    def __init__(self, cfgs, image_dim, device, lazy_count=False):
        super().__init__()
        self.height, self.width = image_dim
        self.device = device
        self.event_mode = cfgs.event_mode
        self.num_bins = cfgs.num_bins
        self.seq_id = -1
        self.img_id = 0
        self.num_events = -1
        self.event_voxel_grids = None
        self.v2e_net = EventEmulator(output_mode=self.event_mode, num_bins=cfgs.num_bins, pl=cfgs.pl, ps=cfgs.ps,
                                     ql=cfgs.ql, qs=cfgs.qs, pos_thres=cfgs.C, neg_thres=cfgs.C,
                                     sigma_thres=cfgs.threshold_sigma, cutoff_hz=cfgs.cutoff_hz,
                                     refractory_period_s=cfgs.refractory_period_s, leak_rate_hz=0.1,
                                     shot_noise_rate_hz=1, device=device, lazy_count=lazy_count)
        self.e2v_net = CistaLSTCNet(image_dim=image_dim, base_channels=cfgs.base_channels, depth=cfgs.depth,
                                    num_bins=cfgs.num_bins)

    def reset_v2e(self, seq_idx):
        if seq_idx != self.seq_id:
            self.v2e_net.reset()
            self.seq_id = seq_idx
            self.img_id = 0

    def forward(self, inputs, timestamps, pred_img, prev_states, seq_idx):
        if pred_img is None:
            pred_img = torch.zeros_like(inputs[:, 0:1, :, :]).float()
        self.reset_v2e(seq_idx)
        self.img_id += 1
        voxels, n = self.v2e_net(inputs, timestamps)
        self.num_events = n
        self.event_voxel_grids = voxels.clone().detach()
        return self.e2v_net(voxels, pred_img, prev_states)
