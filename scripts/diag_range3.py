"""Diagnostic (GPU): decoder stage (Dg conv + ConvLSTM) with z ~ scale * N(0,1) on sample 1 and
None previous states, against the fp64 oracle, for growing scales."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import fixtures as fx  # noqa: E402
from oracle.cista_oracle import CistaLSTCOracle, relu  # noqa: E402
from tests.test_gpu_numerics import make_model, _nhwc, _nchw, scaled_params  # noqa: E402
from v2e2v_amd import _lib  # noqa: E402

out = open("gpurun_out/diag_range3.txt", "w")
B, h, w, C = 2, 32, 32, 64
for wsc in [1.0, 100.0]:
    params = scaled_params(wsc)
    m = make_model(params)
    packed = m.packed_params()
    ws = m.workspace(B, 2 * h, 2 * w, torch.device("cuda"))
    cfg = _lib.CistaConfig(C, 5, 5)
    L = _lib.lib()
    o = CistaLSTCOracle(params, 5, dtype=np.float64)
    rng = np.random.default_rng(3)
    for scale in [1e4, 1e8, 1e15, 1e20, 1e23]:
        z = rng.standard_normal((B, 2 * C, h, w)) * np.array([1.0, scale]).reshape(B, 1, 1, 1)
        z[rng.random(z.shape) < 0.3] = 0
        hs, cs = torch.empty(B, h, w, C, device="cuda"), torch.empty(B, h, w, C, device="cuda")
        tz = _nhwc(z)
        _lib.check(L.cista_stage_decoder(ctypes.byref(cfg), packed.data_ptr(), B, h, w, tz.data_ptr(), None, None,
                                         hs.data_ptr(), cs.data_ptr(), ws.data_ptr(), ws.numel(), None), "dec")
        torch.cuda.synchronize()
        zd = z.astype(np.float32).astype(np.float64)
        y = relu(o._conv("Dg.conv.conv2d", zd))
        g = o._conv("Dg.recurrent_block.Gates", np.concatenate([y, np.zeros_like(y)], 1))
        rh, rc = o.lstm(y, None)
        gh, gc = _nchw(hs), _nchw(cs)
        d = np.abs(gc - rc)
        i = np.unravel_index(np.argmax(d), d.shape)
        gi = (i[0], 192 + i[1], i[2], i[3])                   # cell gate pre-activation
        print(f"w x{wsc:g} z x{scale:g}: c err {d.max():.3e} at {i} got {gc[i]:.4e} ref {rc[i]:.4e} "
              f"n_bad {(d > 1e-3).sum()} rows {sorted(set(np.argwhere(d > 1e-3)[:, 2].tolist()))[:10]} "
              f"cols {sorted(set(np.argwhere(d > 1e-3)[:, 3].tolist()))[:10]} g_pre {g[gi]:.4e} max|y| {np.abs(y).max():.3e}",
              file=out)
out.close()
print(open("gpurun_out/diag_range3.txt").read())
