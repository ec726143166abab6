"""Dump the upsample conv's q planes of one fixed B=1 input (for comparing library builds)."""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from oracle import fixtures as fx
from v2e2v_amd import CistaLSTCNet, _lib

dev = torch.device("cuda")
H, W, C = 180, 240, 64
h, w = H // 2, W // 2
m = CistaLSTCNet([H, W])
p = fx.stress_params(64, 5, 5, seed=21)
m.load_state_dict(fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in p.items()}, 5))
m = m.to(dev).eval()
packed = m.packed_params()
cfg = _lib.CistaConfig(64, 5, 5)
L = _lib.lib()
g = torch.Generator(device=dev).manual_seed(1)
hp = torch.randn(1, h, w, C, device=dev, generator=g)
ws = torch.zeros(L.cista_workspace_bytes(ctypes.byref(cfg), 1, H, W), dtype=torch.uint8, device=dev)
rec, pre = torch.empty(1, 1, H, W, device=dev), torch.empty(1, 1, H, W, device=dev)
_lib.check(L.cista_stage_output(ctypes.byref(cfg), packed.data_ptr(), 1, h, w, hp.data_ptr(), rec.data_ptr(),
                                pre.data_ptr(), ws.data_ptr(), ws.numel(), None), "out")
torch.cuda.synchronize()
q = ws[256:256 + 9 * H * W * 4].view(torch.float32).cpu().numpy()
np.save(sys.argv[1], q)
print("saved", sys.argv[1])
