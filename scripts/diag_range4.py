"""Diagnostic (GPU): frame 0 of the weights-x100 sequence; the decoder (Dg + ConvLSTM) recomputed in
fp64 from the HIP path's own z, against the HIP h / c (is the error made in the decoder or
inherited from z?)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.cista_oracle import CistaLSTCOracle, relu  # noqa: E402
from tests.test_gpu_numerics import make_model, raw_voxels, scaled_params, _nhwc, _nchw  # noqa: E402
from v2e2v_amd import _lib  # noqa: E402

out = open("gpurun_out/diag_range4.txt", "w")
vox = raw_voxels()
params = scaled_params(100.0)
m = make_model(params)
B, H, W = vox.shape[1], vox.shape[3], vox.shape[4]
with torch.no_grad():
    rec, st = m(torch.from_numpy(vox[0]).cuda(), torch.zeros(B, 1, H, W, device="cuda"), None)
torch.cuda.synchronize()
z = st[1].cpu().numpy().astype(np.float64)
gh, gc = st[2][0].cpu().numpy(), st[2][1].cpu().numpy()
o = CistaLSTCOracle(params, 5, dtype=np.float64)
y = relu(o._conv("Dg.conv.conv2d", z))
g = o._conv("Dg.recurrent_block.Gates", np.concatenate([y, np.zeros_like(y)], 1))
rh, rc = o.lstm(y, None)
for name, a, r in [("h", gh, rh), ("c", gc, rc)]:
    d = np.abs(a - r)
    bad = np.argwhere(d > 1e-2)
    print(f"{name}: max err {d.max():.3e}, n_bad {len(bad)}, first {bad[:8].tolist()}", file=out)
    for b in bad[:4]:
        b = tuple(b)
        gi = (b[0], 192 + b[1], b[2], b[3])
        terms_y = np.abs(y[b[0], :, max(b[2] - 1, 0):b[2] + 2, max(b[3] - 1, 0):b[3] + 2]).max()
        print(f"   at {b}: hip {a[b]:.5e} ref {r[b]:.5e}  g_pre {g[gi]:.4e} i_pre {g[(b[0], b[1], b[2], b[3])]:.4e} "
              f"max|y| nbhd {terms_y:.3e}", file=out)
# the decoder stage on the same z through the C ABI: bit-identical to the module's?
packed = m.packed_params()
ws = m.workspace(B, H, W, torch.device("cuda"))
cfg = _lib.CistaConfig(64, 5, 5)
hs, cs = torch.empty(B, H // 2, W // 2, 64, device="cuda"), torch.empty(B, H // 2, W // 2, 64, device="cuda")
tz = _nhwc(z.astype(np.float32))
_lib.check(_lib.lib().cista_stage_decoder(ctypes.byref(cfg), packed.data_ptr(), B, H // 2, W // 2, tz.data_ptr(), None,
                                          None, hs.data_ptr(), cs.data_ptr(), ws.data_ptr(), ws.numel(), None), "dec")
torch.cuda.synchronize()
print("stage h == module h:", np.array_equal(_nchw(hs), gh), " max diff", np.abs(_nchw(hs) - gh).max(), file=out)
out.close()
print(open("gpurun_out/diag_range4.txt").read())
