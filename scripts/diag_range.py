"""Diagnostic (GPU): the range pass on the LSTC stage with None states -- where do the HIP
results and the fp64 oracle differ?  Writes a summary to gpurun_out/diag_range.txt."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import fixtures as fx  # noqa: E402
from oracle.cista_oracle import CistaLSTCOracle  # noqa: E402
from tests.test_gpu_numerics import make_model, _nhwc, _nchw  # noqa: E402
from v2e2v_amd import _lib  # noqa: E402

out = open("gpurun_out/diag_range.txt", "w")
B, h, w, C = 2, 20, 28, 64
params = fx.stress_params(C, 5, 5, seed=7)
m = make_model(params)
packed = m.packed_params()
ws = m.workspace(B, 2 * h, 2 * w, torch.device("cuda"))
cfg = _lib.CistaConfig(C, 5, 5)
L = _lib.lib()
o = CistaLSTCOracle(params, 5, dtype=np.float64)
rng = np.random.default_rng(21)
for scale in [1.0, 1e3, 1e5, 1e6]:
    x1 = rng.standard_normal((B, C, h, w)) * scale
    for none in [False, True]:
        zp = rng.standard_normal((B, 2 * C, h, w))
        cp = rng.standard_normal((B, 2 * C, h, w))
        z, c = torch.empty(B, h, w, 2 * C, device="cuda"), torch.empty(B, h, w, 2 * C, device="cuda")
        tx, tz, tc = _nhwc(x1), _nhwc(zp), _nhwc(cp)
        _lib.check(L.cista_stage_lstc(ctypes.byref(cfg), packed.data_ptr(), B, h, w, tx.data_ptr(),
                                      None if none else tz.data_ptr(), None if none else tc.data_ptr(),
                                      z.data_ptr(), c.data_ptr(), ws.data_ptr(), ws.numel(), None), "lstc")
        torch.cuda.synchronize()
        x1d = x1.astype(np.float32).astype(np.float64)
        zpd, cpd = zp.astype(np.float32).astype(np.float64), cp.astype(np.float32).astype(np.float64)
        rz, rc = o.lstc(x1d, None, None) if none else o.lstc(x1d, zpd, cpd)
        gz, gc = _nchw(z), _nchw(c)
        for name, g, r in [("z", gz, rz), ("c", gc, rc)]:
            d = np.abs(g - r)
            i = np.unravel_index(np.argmax(d), d.shape)
            print(f"scale {scale:g} none {none} {name}: rel {d.max() / np.abs(r).max():.3e} at {i} got {g[i]:.6e} "
                  f"ref {r[i]:.6e}; frac(|d|>1e-4 max) {np.mean(d > 1e-4 * np.abs(r).max()):.4f}", file=out)
# P0 alone (z0) through the lstc with the gates: compare z0 via c with i = 1 impossible; so also the
# ISTA-free pieces: P0 output = workspace z0 (carve: header 256 + full, x1, z0)
out.close()
print(open("gpurun_out/diag_range.txt").read())
