"""Whole-sequence hipGraph replay of the CISTA-LSTC recurrence (no reference counterpart: the
reference's harness calls ``CistaLSTCNet.forward`` once per frame, test_e2v.py:105-117; this is
the same loop with its ~21 x L kernel launches captured once, include/cista_lstc.h
``cista_sequence_*``).

``CistaSequence(model, voxels)`` binds a device buffer of L voxel frames (L, B, nb, H, W);
``run()`` replays the L recurrent frames -- prev_image = previous output, states carried, the
first frame from ``prev_image`` (zeros by default) and ``prev_states`` (None by default) --
with one graph launch, and returns (recs (L, B, 1, H, W), states of the last frame).  Refill
``voxels`` in place and call ``run()`` again for the next sequence: every pointer is baked into
the graph, nothing is re-launched from Python.  The parameters are re-packed and the graph
re-captured automatically when they change (optimizer step, load_state_dict).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


class CistaSequence:
    def __init__(self, model, voxels: torch.Tensor, prev_image: torch.Tensor | None = None,
                 prev_states=None):
        if voxels.dim() != 5 or not voxels.is_cuda or voxels.dtype != torch.float32 or not voxels.is_contiguous():
            raise ValueError("voxels must be a contiguous float32 CUDA tensor (L, B, num_bins, H, W)")
        L, B, nb, H, W = voxels.shape
        if nb != model.num_bins or H % 2 or W % 2:
            raise ValueError(f"voxels {tuple(voxels.shape)} do not fit the model (num_bins={model.num_bins}, even H, W)")
        self.model, self.voxels = model, voxels
        self.L, self.B, self.H, self.W = L, B, H, W
        dev, C, h, w, cl = voxels.device, model.base_channels, H // 2, W // 2, torch.channels_last
        self.recs = torch.empty(L, B, 1, H, W, device=dev)
        self.prev0 = torch.zeros(B, 1, H, W, device=dev) if prev_image is None else prev_image.detach().float().contiguous()
        mk = lambda c: torch.empty(B, c, h, w, device=dev, memory_format=cl)   # noqa: E731
        self.sets = [[mk(2 * C), mk(2 * C), mk(C), mk(C)] for _ in range(2)]    # ping-pong state sets
        if prev_states is None:
            self.init = [None] * 4
        else:
            hc = prev_states[-1]
            self.init = [t.detach().float().contiguous(memory_format=cl) if t is not None else None
                         for t in (prev_states[0], prev_states[-2], None if hc is None else hc[0],
                                   None if hc is None else hc[1])]
        self._seq = None
        self._packed = None

    def _io(self):
        P = _lib.ptr
        ios = (_lib.CistaFrameIO * self.L)()
        for f in range(self.L):
            prev = self.prev0 if f == 0 else self.recs[f - 1]
            pst = self.init if f == 0 else self.sets[(f - 1) % 2]
            out = self.sets[f % 2]
            ios[f] = _lib.CistaFrameIO(P(self.voxels[f]), P(prev), P(pst[0]), P(pst[1]), P(pst[2]), P(pst[3]),
                                       P(self.recs[f]), P(out[0]), P(out[1]), P(out[2]), P(out[3]))
        return ios

    def _capture(self):
        self.close()
        m = self.model
        self._packed = m.packed_params()
        self._ws = m.workspace(self.B, self.H, self.W, self.voxels.device)
        handle = ctypes.c_void_p()
        L = _lib.lib()
        # the library orders its capture stream after torch's current stream (inputs, packing)
        _lib.check(L.cista_sequence_capture(ctypes.byref(m._cfg()), self._packed.data_ptr(), self.B, self.H, self.W,
                                            self._io(), self.L, self._ws.data_ptr(), self._ws.numel(),
                                            ctypes.byref(handle), _lib.stream_handle(self.voxels.device)),
                   "cista_sequence_capture")
        self._seq = handle

    def run(self):
        """One replay of the L-frame recurrence on torch's current stream."""
        if self._seq is None or self.model.packed_params() is not self._packed:
            self._capture()
        dev = self.voxels.device
        _lib.check(_lib.lib().cista_sequence_launch(self._seq, _lib.stream_handle(dev)), "cista_sequence_launch")
        last = self.sets[(self.L - 1) % 2]
        return self.recs, [last[0], last[1], (last[2], last[3])]

    def close(self):
        if self._seq is not None:
            _lib.lib().cista_sequence_destroy(self._seq)
            self._seq = None

    def __del__(self):
        try:
            self.close()
        except Exception:       # interpreter shutdown: the library may be gone
            pass
