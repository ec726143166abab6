"""Diagnostic (GPU): full CistaLSTCNet frames with weights x100 (activations up to 1e23): per frame
and per output tensor, the error of the HIP path and of the fp32 CPU reference against fp64."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.cista_oracle_torch import CistaLSTCTorchCPU  # noqa: E402
from tests.conftest import rel_err  # noqa: E402
from tests.test_gpu_numerics import make_model, raw_voxels, scaled_params  # noqa: E402

out = open("gpurun_out/diag_range2.txt", "w")
wscale = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
vox = raw_voxels()
params = scaled_params(wscale)
m = make_model(params)
r32 = CistaLSTCTorchCPU(params, 5)
r64 = CistaLSTCTorchCPU(params, 5, dtype=torch.float64)
B, H, W = vox.shape[1], vox.shape[3], vox.shape[4]
prev = torch.zeros(B, 1, H, W, device="cuda")
st = None
p32 = torch.zeros(B, 1, H, W)
p64 = torch.zeros(B, 1, H, W, dtype=torch.float64)
s32 = s64 = None
flat = lambda s: [s[0], s[1], s[2][0], s[2][1]]   # noqa: E731
with torch.no_grad():
    for f in range(vox.shape[0]):
        # every path from the SAME fp64-truth inputs of this frame (no error carried over)
        ev = torch.from_numpy(vox[f])
        gin = None if s64 is None else [t.float().cuda().contiguous() if not isinstance(t, tuple) else
                                        tuple(u.float().cuda().contiguous() for u in t) for t in s64]
        g_rec, g_st = m(ev.cuda(), p64.float().cuda(), gin)
        c_in = None if s64 is None else [t.float() if not isinstance(t, tuple) else tuple(u.float() for u in t)
                                         for t in s64]
        o32, n32 = r32.forward(ev, p64.float(), c_in)
        o64, n64 = r64.forward(ev.double(), p64, s64)
        for name, g, a, t in zip(["rec", "c_lstc", "z", "h", "c"], [g_rec] + flat(g_st), [o32] + flat(n32),
                                 [o64] + flat(n64)):
            g, a, t = g.cpu().double().numpy(), a.double().numpy(), t.double().numpy()
            d = np.abs(g - t)
            i = np.unravel_index(np.argmax(d), d.shape)
            print(f"frame {f} {name:7s} hip {rel_err(g, t):.3e} ref32 {rel_err(a, t):.3e}  max|t| {np.abs(t).max():.3e}"
                  f"  worst {i} hip {g[i]:.6e} truth {t[i]:.6e} ref32 {a[i]:.6e}", file=out)
        p64, s64 = o64, n64
out.close()
print(open("gpurun_out/diag_range2.txt").read())
