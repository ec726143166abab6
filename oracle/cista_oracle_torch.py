"""PyTorch-CPU op-for-op restatement of the reference CISTA-LSTC forward.

TEST INFRASTRUCTURE ONLY, like oracle/cista_oracle.py (the numpy oracle).  Nothing in the
product package (``v2e2v_amd``) imports this file.  Its one job is ``bench.py``'s
``cpu_baseline`` leg: the reference's own CPU path is ATen's CPU kernels (oneDNN convolutions,
multi-threaded), so timing the same ops here gives the baseline the GPU number is quoted
against ("kind": "port").  The numpy oracle stays the parity checker; this one is pinned to
the same golden vectors by ``tests/test_oracle_golden.py``.

Every step cites the reference file:line it restates.  Layout NCHW, fp32 (or fp64), on CPU.
Parameters: a dict of UNIQUE tensors keyed as ``oracle.fixtures.param_shapes`` ('lista.*' is
the tied IstaBlock), the same dict the numpy oracle takes.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


class CistaLSTCTorchCPU:
    """CistaLSTCNet.forward (reference e2v/e2v_model.py:41-90) as ATen CPU calls."""

    def __init__(self, params: dict, depth: int = 5, dtype=torch.float32, requires_grad: bool = False):
        self.p = {k: torch.as_tensor(np.asarray(v)).to(dtype).requires_grad_(requires_grad)
                  for k, v in params.items()}
        self.depth = depth
        self.dtype = dtype
        self.C = self.p["W0.conv2d.weight"].shape[0]

    def _conv(self, name, x, stride=1, pad=True):
        """Conv2d(k=3, padding=1, padding_mode='reflect') (base_layers.py:140, :48-50, :88);
        pad=False is the upsample conv after its own ReflectionPad2d (:178-180)."""
        if pad:
            x = F.pad(x, (1, 1, 1, 1), mode="reflect")
        return F.conv2d(x, self.p[name + ".weight"], self.p[name + ".bias"], stride=stride)

    def lstc(self, x1, z_prev, c_prev):
        """ConvLSTC.forward (base_layers.py:52-71)."""
        B, _, h, w = x1.shape
        if z_prev is None:                                                   # :54-55
            z_prev = x1.new_zeros(B, 2 * self.C, h, w)
        i_g, f_g = self._conv("P0.gates", torch.cat([x1, z_prev], 1)).chunk(2, 1)   # :57-58
        i_g, f_g = torch.sigmoid(i_g), torch.sigmoid(f_g)                    # :59-60
        z0 = self._conv("P0.P0", x1)                                         # :61
        o_g = torch.sigmoid(self._conv("P0.out_gates", torch.cat([z0, z_prev], 1)))  # :63
        if c_prev is None:                                                   # :65-66
            c_prev = torch.zeros_like(z0)
        c = f_g * c_prev + i_g * z0                                          # :67
        return o_g * torch.tanh(c), c                                        # :69-71

    def lstm(self, x, state):
        """ConvLSTM.forward (base_layers.py:90-130), gates (in, remember, out, cell) :116."""
        if state is None:                                                    # :97-107
            z = x.new_zeros(x.shape[0], self.C, *x.shape[2:])
            state = (z, z)
        h_prev, c_prev = state
        gi, gr, go, gc = self._conv("Dg.recurrent_block.Gates",
                                    torch.cat([x, h_prev], 1)).chunk(4, 1)   # :112-116
        c = torch.sigmoid(gr) * c_prev + torch.sigmoid(gi) * torch.tanh(gc)  # :119-127
        return torch.sigmoid(go) * torch.tanh(c), c                          # :128

    def forward(self, events, prev_image, prev_states=None):
        with torch.no_grad():
            return self.forward_grad(events, prev_image, prev_states)

    def forward_grad(self, events, prev_image, prev_states=None):
        """The same forward under autograd (the CPU baseline of the BPTT training step)."""
        if prev_states is None:                                              # e2v_model.py:57-58
            prev_states = [None, None, None]
        x_e = self._conv("We.conv2d", events)                                # :62
        x_i = self._conv("Wi.conv2d", prev_image)                            # :63
        x1 = self._conv("W0.conv2d", torch.cat([x_e, x_i], 1), stride=2)     # :64-66
        z, c_lstc = self.lstc(x1, prev_states[-2], prev_states[0])           # :68
        lam = self.p["lista.Lambda"]
        for _ in range(self.depth):                                          # :72-78 (tied)
            x = self._conv("lista.P.conv2d", x1 - self._conv("lista.D.conv2d", z)) + z
            z = torch.relu(x - lam) - torch.relu(-x - lam)                   # base_layers.py:11-12
        y = torch.relu(self._conv("Dg.conv.conv2d", z))                      # base_layers.py:221-225
        h, c = self.lstm(y, prev_states[-1])
        up = F.interpolate(h, size=(2 * h.shape[2], 2 * h.shape[3]), mode="bilinear",
                           align_corners=False)                              # base_layers.py:198
        u = torch.relu(self._conv("upsamp_conv.conv2d", F.pad(up, (1, 1, 1, 1), mode="reflect"),
                                  pad=False))                                # :178-180, :208-210
        rec = torch.sigmoid(self._conv("final_conv.conv2d", u))              # e2v_model.py:87-88
        return rec, [c_lstc, z, (h, c)]

    def run_sequence(self, voxels, prev_image=None):
        """voxels [F,B,nb,H,W] (numpy or tensor); prev_image starts at zeros and is the previous
        output (reference test_e2v.py:110-117).  Returns numpy (recs [F,B,1,H,W], states)."""
        v = torch.as_tensor(np.asarray(voxels)).to(self.dtype)
        F_, B, _, H, W = v.shape
        prev = torch.zeros(B, 1, H, W, dtype=self.dtype) if prev_image is None else prev_image
        states = None
        recs = []
        for f in range(F_):
            prev, states = self.forward(v[f], prev, states)
            recs.append(prev)
        st = [states[0].numpy(), states[1].numpy(), (states[2][0].numpy(), states[2][1].numpy())]
        return torch.stack(recs).numpy(), st


def bptt_step(net: CistaLSTCTorchCPU, voxels, target):
    """One train_e2v.py:108-130 step on the CPU restatement (bench.py's training cpu_baseline):
    L recurrent frames, prev_img = output.clone() (not detached), L1 on the last frame, one
    backward through the whole sequence; returns the loss."""
    v = torch.as_tensor(np.asarray(voxels)).to(net.dtype)
    F_, B, _, H, W = v.shape
    prev = torch.zeros(B, 1, H, W, dtype=net.dtype)
    states = None
    for f in range(F_):
        out, states = net.forward_grad(v[f], prev, states)
        prev = out.clone()
    loss = torch.nn.functional.l1_loss(out, torch.as_tensor(np.asarray(target)).to(net.dtype))
    for t in net.p.values():
        t.grad = None
    loss.backward()
    return float(loss.item())
