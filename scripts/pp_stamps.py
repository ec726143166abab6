"""Segment timeline of the two-tile ISTA convs from a CISTA_STAMPS=1 diagnostic build
(cista_pingpong.hpp PP_STAMP): per half (waves 0-3 / 4-7), the median shader cycles of each
K-chunk's work, its barrier wait, the epilogue's parts and its barrier wait, for the third tile
of every half-slot.

usage: CISTA_HIP_LIB=v2e2v_amd/variants/stamps.so python scripts/pp_stamps.py [B] [layer ...]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402


def analyse(st, name, nch):
    st = st.reshape(-1, 8, 24).astype(np.int64)
    out = {"layer": name}
    for half in (0, 1):
        s = st[:, 4 * half:4 * half + 4].reshape(-1, 24)
        s = s[s[:, 1] != 0]
        if not len(s):
            continue
        q = lambda x: int(np.median(x))      # noqa: E731
        seg = {}
        ngrp = (nch + 1) // 2
        prev = s[:, 1]
        for g in range(min(ngrp, 2)):
            # K segment g: work, barrier wait; memory segment g: work, barrier wait
            seg[f"k{g}_work"] = q(s[:, 2 + 4 * g] - prev)
            seg[f"k{g}_wait"] = q(s[:, 3 + 4 * g] - s[:, 2 + 4 * g])
            seg[f"m{g}_work"] = q(s[:, 4 + 4 * g] - s[:, 3 + 4 * g])
            seg[f"m{g}_wait"] = q(s[:, 5 + 4 * g] - s[:, 4 + 4 * g])
            prev = s[:, 5 + 4 * g]
        last = 4 * (ngrp - 1) if ngrp <= 2 else None
        if last is not None:
            seg["epi_aux_issue"] = q(s[:, 12] - s[:, 3 + last])
            seg["epi_math"] = q(s[:, 13] - s[:, 12])
            seg["epi_halo_and_stores"] = q(s[:, 14] - s[:, 13])
            seg["commit"] = q(s[:, 4 + last] - s[:, 14])
        seg["tile_total"] = q(s[:, 5 + 4 * (min(ngrp, 2) - 1)] - s[:, 1])
        clk = np.median((s[:, 4 + last if last is not None else 4] - s[:, 1])
                        / np.maximum(1, s[:, 17] - s[:, 16]) * 100.0)
        seg["clock_mhz"] = int(clk)
        seg["waves"] = int(len(s))
        out[f"half{half}"] = seg
    return out


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    names = sys.argv[2:] or ["ista_D", "ista_P"]
    H, W = 180, 240
    dev = torch.device("cuda", 0)
    m = CistaLSTCNet([H, W])
    bench.he_init_(torch, m, 7)
    m = m.to(dev).eval()
    L = _lib.lib()
    L.cista_debug_set_stamps.argtypes = [ctypes.c_void_p]
    vox = bench.synth_voxels(torch, 2, B, 5, H, W, 15000, 1, dev)
    buf = torch.zeros(24 << 17, dtype=torch.int64, device=dev)
    C = m.base_channels
    h, w = H // 2, W // 2
    cl = torch.channels_last
    with torch.no_grad():
        rec0, st0 = m(vox[0], torch.zeros(B, 1, H, W, device=dev), None)
        outs = [torch.empty(B, 1, H, W, device=dev), torch.empty(B, 2 * C, h, w, device=dev, memory_format=cl),
                torch.empty(B, 2 * C, h, w, device=dev, memory_format=cl),
                torch.empty(B, C, h, w, device=dev, memory_format=cl),
                torch.empty(B, C, h, w, device=dev, memory_format=cl)]
        ws = m.workspace(B, H, W, dev)
        packed = m.packed_params()
        ev = vox[1].contiguous()
        io = _lib.CistaFrameIO(ev.data_ptr(), rec0.data_ptr(), st0[0].data_ptr(), st0[1].data_ptr(),
                               st0[2][0].data_ptr(), st0[2][1].data_ptr(), *[o.data_ptr() for o in outs])
        cfg = m._cfg()
        s = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(L.cista_forward(ctypes.byref(cfg), packed.data_ptr(), B, H, W, ctypes.byref(io),
                                   ws.data_ptr(), ws.numel(), s), "forward")
        for name in names:
            lid = _lib.LAYERS.index(name)
            run = lambda: _lib.check(L.cista_launch_layer(ctypes.byref(cfg), packed.data_ptr(), lid, B, H, W,  # noqa: E731
                                                         ctypes.byref(io), ws.data_ptr(), ws.numel(), s), name)
            for _ in range(20):
                run()
            buf.zero_()
            torch.cuda.synchronize()
            L.cista_debug_set_stamps(ctypes.c_void_p(buf.data_ptr()))
            run()
            torch.cuda.synchronize()
            L.cista_debug_set_stamps(ctypes.c_void_p(0))
            nch = 4 if name == "ista_D" else 2
            print(json.dumps(analyse(buf[:256 * 8 * 24].cpu().numpy(), name, nch)), flush=True)


if __name__ == "__main__":
    main()
