"""Which frame stage gives different bits for one sample run alone (B=1) and inside a batch?
Each stage entry (include/cista_lstc.h) gets the same random inputs at B=Bb and at B=1.
usage: python scripts/diag_batch_bits.py [Bb]"""
import ctypes
import sys
import os
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
Bb = int(sys.argv[1]) if len(sys.argv) > 1 else 12
R = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
ev, img = R(Bb, 5, H, W), torch.rand(Bb, 1, H, W, device=dev, generator=g)
x1, zp, cp = R(Bb, h, w, C), R(Bb, h, w, 2 * C), R(Bb, h, w, 2 * C)
hp, cpp = R(Bb, h, w, C), R(Bb, h, w, C)


def run(B):
    ws = torch.empty(L.cista_workspace_bytes(ctypes.byref(cfg), B, H, W), dtype=torch.uint8, device=dev)
    o = {}
    o["x1"] = torch.empty(B, h, w, C, device=dev)
    _lib.check(L.cista_stage_input(ctypes.byref(cfg), packed.data_ptr(), B, H, W, ev[:B].data_ptr(), img[:B].data_ptr(),
                                   o["x1"].data_ptr(), ws.data_ptr(), ws.numel(), None), "in")
    o["z"], o["c"] = torch.empty(B, h, w, 2 * C, device=dev), torch.empty(B, h, w, 2 * C, device=dev)
    _lib.check(L.cista_stage_lstc(ctypes.byref(cfg), packed.data_ptr(), B, h, w, x1[:B].data_ptr(), zp[:B].data_ptr(),
                                  cp[:B].data_ptr(), o["z"].data_ptr(), o["c"].data_ptr(), ws.data_ptr(), ws.numel(), None), "lstc")
    o["zi"] = zp[:B].clone()
    _lib.check(L.cista_stage_ista(ctypes.byref(cfg), packed.data_ptr(), B, h, w, x1[:B].data_ptr(), o["zi"].data_ptr(), 5,
                                  ws.data_ptr(), ws.numel(), None), "ista")
    o["hh"], o["cc"] = torch.empty(B, h, w, C, device=dev), torch.empty(B, h, w, C, device=dev)
    _lib.check(L.cista_stage_decoder(ctypes.byref(cfg), packed.data_ptr(), B, h, w, zp[:B].data_ptr(), hp[:B].data_ptr(),
                                     cpp[:B].data_ptr(), o["hh"].data_ptr(), o["cc"].data_ptr(), ws.data_ptr(), ws.numel(), None), "dec")
    o["rec"], o["pre"] = torch.empty(B, 1, H, W, device=dev), torch.empty(B, 1, H, W, device=dev)
    _lib.check(L.cista_stage_output(ctypes.byref(cfg), packed.data_ptr(), B, h, w, hp[:B].data_ptr(), o["rec"].data_ptr(),
                                    o["pre"].data_ptr(), ws.data_ptr(), ws.numel(), None), "out")
    torch.cuda.synchronize()
    return o


a, b = run(Bb), run(1)
for k in a:
    d = (a[k][:1] - b[k]).abs().max().item()
    print(f"{k:4s} bit-equal={torch.equal(a[k][:1], b[k])} maxdiff={d:.3e} scale={a[k][:1].abs().max().item():.3e}")


# the upsample conv alone: q planes (B, 9, H, W) fp32 at workspace offset 256 (WS_HEADER)
def q_planes(B):
    ws = torch.zeros(L.cista_workspace_bytes(ctypes.byref(cfg), B, H, W), dtype=torch.uint8, device=dev)
    rec, pre = torch.empty(B, 1, H, W, device=dev), torch.empty(B, 1, H, W, device=dev)
    _lib.check(L.cista_stage_output(ctypes.byref(cfg), packed.data_ptr(), B, h, w, hp[:B].data_ptr(), rec.data_ptr(),
                                    pre.data_ptr(), ws.data_ptr(), ws.numel(), None), "out")
    torch.cuda.synchronize()
    return ws[256:256 + B * 9 * H * W * 4].view(torch.float32).view(B, 9, H, W)


qa, qb = q_planes(Bb), q_planes(1)
diff = (qa[:1] - qb).abs()
print("q bit-equal", torch.equal(qa[:1], qb), "maxdiff", diff.max().item())
nz = (diff > 0).nonzero()
print("differing elements", nz.shape[0], "of", diff.numel())
if nz.shape[0]:
    ys, xs = nz[:, 2], nz[:, 3]
    print("taps", torch.unique(nz[:, 1]).tolist()[:9], "rows", ys.min().item(), ys.max().item(),
          "cols", xs.min().item(), xs.max().item())
    print("row histogram (first 20)", torch.bincount(ys, minlength=H)[:20].tolist())
    print("col histogram (first 20)", torch.bincount(xs, minlength=W)[:20].tolist())
