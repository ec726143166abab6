"""Phase timeline of the conv kernels from a CISTA_STAMPS=1 diagnostic build.

usage: CISTA_HIP_LIB=v2e2v_amd/variants/stamps.so python scripts/stamps.py [B] [layer ...]

Every wave's lane 0 records shader-clock timestamps at its phase boundaries (cista_kernels.hpp,
CISTA_STAMP): start, prologue staged, end of each K-chunk, MFMA loop done, epilogue stores issued.
Prints, per layer, the median / p90 cycles of each phase per wave, the in-kernel clock, and how
much of each CU's time had at least one workgroup inside its K loop (the MFMA phase)."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402


def analyse(st, name):
    st = st.reshape(-1, 24).astype(np.int64)
    st = st[st[:, 1] != 0]
    hw, xcc = st[:, 0] & 0xFFFFFFFF, st[:, 0] >> 32
    cu = (xcc << 16) | (((hw >> 13) & 7) << 8) | ((hw >> 8) & 15)      # xcc, se, cu
    t0, tpro, tloop, tend = st[:, 1], st[:, 2], st[:, 11], st[:, 12]
    nchunk = int(np.max(np.sum(st[:, 3:11] != 0, axis=1)))
    chunks = [st[:, 3 + k] - (st[:, 2 + k] if k else tpro) for k in range(nchunk)]
    clk = float(np.median((tend - t0) / np.maximum(1, st[:, 14] - st[:, 13]) * 100.0))   # MHz
    q = lambda x: (int(np.median(x)), int(np.percentile(x, 90)))   # noqa: E731
    out = {"layer": name, "waves": int(len(st)), "clock_mhz": round(clk), "k_chunks": nchunk,
           "prologue": q(tpro - t0), "chunks": [q(c) for c in chunks], "loop_tail": q(tloop - st[:, 2 + nchunk]),
           "epilogue": q(tend - tloop), "epi_sync": q(st[:, 15] - tloop), "epi_math": q(st[:, 16] - st[:, 15]),
           "epi_stores": q(tend - st[:, 16]), "total": q(tend - t0)}
    # per CU: fraction of the CU's busy span during which >= 1 wave is inside its K loop, and
    # during which >= 1 wave is in its prologue / epilogue (memory phases)
    span = tot_loop = tot_mem = tot_both = 0
    for c in np.unique(cu):
        sel = cu == c
        a, p, l, e = t0[sel], tpro[sel], tloop[sel], tend[sel]
        lo, hi = int(a.min()), int(e.max())
        grid = np.zeros((3, (hi - lo) // 64 + 2), np.int32)
        for x0, x1, row in ((p, l, 0), (a, p, 1), (l, e, 1)):
            for u, v in zip((x0 - lo) // 64, (x1 - lo) // 64):
                grid[row, u:v + 1] += 1
        busy = (grid[0] > 0) | (grid[1] > 0)
        span += busy.sum()
        tot_loop += (grid[0] > 0).sum()
        tot_mem += (grid[1] > 0).sum()
        tot_both += ((grid[0] > 0) & (grid[1] > 0)).sum()
    out["cu_frac_in_loop"] = round(tot_loop / span, 3)
    out["cu_frac_in_prologue_or_epilogue"] = round(tot_mem / span, 3)
    out["cu_frac_overlapped"] = round(tot_both / span, 3)
    return out


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    names = sys.argv[2:] or ["ista_D", "ista_P", "gates"]
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
            for _ in range(20):          # warm the clock
                run()
            buf.zero_()
            torch.cuda.synchronize()
            L.cista_debug_set_stamps(ctypes.c_void_p(buf.data_ptr()))
            run()
            torch.cuda.synchronize()
            L.cista_debug_set_stamps(ctypes.c_void_p(0))
            print(json.dumps(analyse(buf.cpu().numpy(), name)), flush=True)


if __name__ == "__main__":
    main()
