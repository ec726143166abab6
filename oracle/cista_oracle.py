"""CPU restatement (numpy) of the reference CISTA-LSTC forward -- the parity ORACLE.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (``v2e2v_amd``) imports this file;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and
only as the checker / the timed CPU baseline ("kind": "port"), never as the thing measured.

Pinned: ``tests/test_oracle_golden.py`` checks this restatement against golden vectors produced
by running the real reference (``/root/reference/e2v``) in the build container
(``tests/golden/make_golden.py``).

Every function cites the reference file:line whose behaviour it restates.  Layout is NCHW
(numpy arrays), dtype float32 (or float64 for the truth shadow).  Convolutions are
reflect-padded 3x3 implemented as im2col + one GEMM.
"""
from __future__ import annotations

import numpy as np


# --------------------------------------------------------------------------------------------
# primitive ops
# --------------------------------------------------------------------------------------------
def reflect_pad1(x: np.ndarray) -> np.ndarray:
    """padding_mode='reflect', padding=1 (torch semantics: index -1 -> 1, H -> H-2).
    Used by every ConvLayer / ConvLSTC / ConvLSTM conv (reference e2v/base_layers.py:48-50,88,140)
    and by ReflectionPad2d(1) (base_layers.py:178)."""
    return np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1)), mode="reflect")


def conv3x3(x: np.ndarray, w: np.ndarray, b: np.ndarray | None, stride: int = 1,
            pad: bool = True) -> np.ndarray:
    """nn.Conv2d(k=3, padding=1 if pad else 0, padding_mode='reflect', stride) on NCHW input.
    (reference e2v/base_layers.py:140 ConvLayer.conv2d; :48-50 ConvLSTC; :88 ConvLSTM; :180)."""
    if pad:
        x = reflect_pad1(x)
    B, Ci, Hp, Wp = x.shape
    Co = w.shape[0]
    Ho = (Hp - 3) // stride + 1
    Wo = (Wp - 3) // stride + 1
    cols = np.empty((B, Ho, Wo, Ci, 3, 3), dtype=x.dtype)
    for ky in range(3):
        for kx in range(3):
            cols[..., ky, kx] = x[:, :, ky:ky + stride * (Ho - 1) + 1:stride,
                                  kx:kx + stride * (Wo - 1) + 1:stride].transpose(0, 2, 3, 1)
    out = cols.reshape(B * Ho * Wo, Ci * 9) @ w.reshape(Co, Ci * 9).T.astype(x.dtype)
    if b is not None:
        out = out + b.astype(x.dtype)
    return np.ascontiguousarray(out.reshape(B, Ho, Wo, Co).transpose(0, 3, 1, 2))


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def relu(x):
    return np.maximum(x, 0)


def softshrink(x, lam):
    """relu(x - lambda) - relu(-x - lambda), literally (reference e2v/base_layers.py:11-12);
    differs from F.softshrink when lambda < 0."""
    return relu(x - lam) - relu(-x - lam)


def upsample_bilinear2x(x: np.ndarray) -> np.ndarray:
    """F.interpolate(size=(2h, 2w), mode='bilinear', align_corners=False)
    (reference e2v/base_layers.py:198): src = (dst + 0.5) * (in/out) - 0.5 clamped at 0,
    upper neighbour clamped to in-1."""
    B, C, h, w = x.shape

    def axis(n_in, n_out):
        scale = np.float32(n_in) / np.float32(n_out)
        d = np.arange(n_out, dtype=np.float32)
        s = np.maximum((d + np.float32(0.5)) * scale - np.float32(0.5), np.float32(0))
        i0 = np.floor(s).astype(np.int64)
        i0 = np.minimum(i0, n_in - 1)
        i1 = np.minimum(i0 + 1, n_in - 1)
        l1 = (s - i0).astype(x.dtype)
        l0 = (1 - l1).astype(x.dtype)
        return i0, i1, l0, l1

    y0, y1, ly0, ly1 = axis(h, 2 * h)
    x0, x1, lx0, lx1 = axis(w, 2 * w)
    # torch order: h0l * (w0l * x00 + w1l * x01) + h1l * (w0l * x10 + w1l * x11)
    horiz = x[:, :, :, x0] * lx0 + x[:, :, :, x1] * lx1
    return horiz[:, :, y0, :] * ly0[None, None, :, None] + horiz[:, :, y1, :] * ly1[None, None, :, None]


# --------------------------------------------------------------------------------------------
# model
# --------------------------------------------------------------------------------------------
class CistaLSTCOracle:
    """Restates CistaLSTCNet (reference e2v/e2v_model.py:5-90) over a dict of UNIQUE parameters
    (keys as oracle.fixtures.param_shapes: 'lista.*' = the tied IstaBlock)."""

    def __init__(self, params: dict, depth: int = 5, dtype=np.float32):
        self.p = {k: np.asarray(v, dtype=dtype) for k, v in params.items()}
        self.depth = depth
        self.dtype = dtype
        self.C = self.p["W0.conv2d.weight"].shape[0]

    def _conv(self, name, x, stride=1, pad=True):
        return conv3x3(x, self.p[name + ".weight"], self.p[name + ".bias"], stride, pad)

    def lstc(self, x1, z_prev, c_prev):
        """ConvLSTC.forward (reference e2v/base_layers.py:52-71)."""
        B, _, h, w = x1.shape
        if z_prev is None:                                              # :54-55
            z_prev = np.zeros((B, 2 * self.C, h, w), self.dtype)
        gates = self._conv("P0.gates", np.concatenate([x1, z_prev], 1))  # :57
        i_g, f_g = np.split(gates, 2, axis=1)                           # :58
        i_g, f_g = sigmoid(i_g), sigmoid(f_g)                           # :59-60
        z0 = self._conv("P0.P0", x1)                                    # :61
        o_g = sigmoid(self._conv("P0.out_gates", np.concatenate([z0, z_prev], 1)))  # :63
        if c_prev is None:                                              # :65-66
            c_prev = np.zeros_like(z0)
        c = f_g * c_prev + i_g * z0                                     # :67
        return o_g * np.tanh(c), c                                      # :69-71

    def lstm(self, x, state):
        """ConvLSTM.forward (reference e2v/base_layers.py:90-130); gate order (in, remember,
        out, cell) :116."""
        if state is None:                                               # :97-107
            z = np.zeros((x.shape[0], self.C) + x.shape[2:], self.dtype)
            state = (z, z)
        h_prev, c_prev = state
        g = self._conv("Dg.recurrent_block.Gates", np.concatenate([x, h_prev], 1))  # :112-113
        gi, gr, go, gc = np.split(g, 4, axis=1)
        c = sigmoid(gr) * c_prev + sigmoid(gi) * np.tanh(gc)            # :119-127
        h = sigmoid(go) * np.tanh(c)                                    # :128
        return h, c

    def forward(self, events, prev_image, prev_states=None, trace: dict | None = None):
        """CistaLSTCNet.forward (reference e2v/e2v_model.py:41-90).  Returns
        (rec_I (B,1,H,W), [c_lstc, z, (h, c)])."""
        dt = self.dtype
        events = np.asarray(events, dt)
        prev_image = np.asarray(prev_image, dt)
        if prev_states is None:                                         # :57-58
            prev_states = [None, None, None]
        x_e = self._conv("We.conv2d", events)                           # :62
        x_i = self._conv("Wi.conv2d", prev_image)                       # :63
        x1 = self._conv("W0.conv2d", np.concatenate([x_e, x_i], 1), stride=2)  # :64-66
        z, c_lstc = self.lstc(x1, prev_states[-2], prev_states[0])      # :68
        if trace is not None:
            trace.update(x_E=x_e, x_I=x_i, x1=x1, z_lstc=z, c_lstc=c_lstc, ista=[])
        lam = self.p["lista.Lambda"]
        tmp = z
        for _ in range(self.depth):                                     # :72-78 (tied block)
            tmp = self._conv("lista.D.conv2d", tmp)
            x = x1 - tmp
            x = self._conv("lista.P.conv2d", x)
            x = x + z
            z = softshrink(x, lam)
            tmp = z
            if trace is not None:
                trace["ista"].append(z)
        y = relu(self._conv("Dg.conv.conv2d", z))                       # base_layers.py:221-225
        h, c = self.lstm(y, prev_states[-1])
        u = relu(self._conv("upsamp_conv.conv2d", reflect_pad1(upsample_bilinear2x(h)),
                            pad=False))                                 # base_layers.py:193-210
        pre = self._conv("final_conv.conv2d", u)                        # e2v_model.py:87
        rec = sigmoid(pre)                                              # :88
        if trace is not None:
            trace.update(dg_y=y, h=h, c=c, u=u, pre_sigmoid=pre)
        return rec.astype(dt), [c_lstc, z, (h, c)]

    def run_sequence(self, voxels, prev_image=None):
        """voxels [F,B,nb,H,W]; prev_image starts at zeros and is the previous output
        (reference test_e2v.py:110-117)."""
        F_, B, _, H, W = voxels.shape
        prev = np.zeros((B, 1, H, W), self.dtype) if prev_image is None else prev_image
        states = None
        recs = []
        for f in range(F_):
            prev, states = self.forward(voxels[f], prev, states)
            recs.append(prev)
        return np.stack(recs), states
