"""Phase timeline of the training dgrad convs (STAGE_ZP2 + EPI_FOLD) from a CISTA_STAMPS=1 build.

usage: CISTA_HIP_LIB=v2e2v_amd/variants/stamps.so python scripts/dgrad_stamps.py [B] [frames]

One BPTT backward at 180x240 (batch B, default 8 as train_e2v.py) runs with the fold-stamp ring on
(cista_debug_set_fold_stamps): every EPI_FOLD launch gets its own region, so the launches of the
backward can be told apart (launch order = the backward's order, last frame first).  Prints one
JSON line per launch: workgroups, K-chunks, the launch's span and each wave's phases (median / p90
shader cycles), the workgroups' start offsets (us; one dispatch round: all start together) and the
waves per CU."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402

WG_MAX, SLOTS = 2048, 24


def summarise(reg):
    st = reg.reshape(-1, SLOTS).astype(np.int64)
    st = st[st[:, 1] != 0]
    if not len(st):
        return None
    hw, xcc = st[:, 0] & 0xFFFFFFFF, st[:, 0] >> 32
    cu = (xcc << 16) | (((hw >> 13) & 7) << 8) | ((hw >> 8) & 15)
    t0, tpro, tloop, tend = st[:, 1], st[:, 2], st[:, 11], st[:, 12]
    nchunk = int(np.max(np.sum(st[:, 3:11] != 0, axis=1)))
    chunks = [st[:, 3 + k] - (st[:, 2 + k] if k else tpro) for k in range(nchunk)]
    q = lambda x: (int(np.median(x)), int(np.percentile(x, 90)))   # noqa: E731
    # launch-level times from the constant 100 MHz clock (s_memrealtime, common to the chip;
    # s_memtime is not synchronised across CUs): workgroup start offsets and the launch's span
    r0, r1 = st[:, 13], st[:, 14]
    rel = (r0 - r0.min()) / 100.0                                     # us
    span_us = float((r1.max() - r0.min()) / 100.0)
    clk = float(np.median((tend - t0) / np.maximum(1, r1 - r0) * 100.0))   # MHz
    _, per_cu = np.unique(cu, return_counts=True)
    return {"waves": int(len(st)), "workgroups": int(len(st) // 4), "k_chunks": nchunk,
            "clock_mhz": round(clk), "launch_span_us": round(span_us, 2),
            "start_offset_us": [round(float(np.median(rel)), 2), round(float(np.percentile(rel, 90)), 2),
                                round(float(rel.max()), 2)],
            "prologue": q(tpro - t0), "chunks": [q(c) for c in chunks], "loop_tail": q(tloop - st[:, 2 + nchunk]),
            "epilogue": q(tend - tloop), "total": q(tend - t0),
            "waves_per_cu": [int(per_cu.min()), int(np.median(per_cu)), int(per_cu.max())], "cus": int(len(per_cu))}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    H, W = 180, 240
    dev = torch.device("cuda", 0)
    m = CistaLSTCNet([H, W])
    bench.he_init_(torch, m, 7)
    m = m.to(dev).train()
    lib = _lib.lib()
    lib.cista_debug_set_fold_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    vox = bench.synth_voxels(torch, L, B, 5, H, W, 15000, 2000, dev)
    target = torch.rand(B, 1, H, W, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    nreg = 24 * L
    buf = torch.zeros(nreg * WG_MAX * 4 * SLOTS, dtype=torch.int64, device=dev)

    def step(stamped):
        prev = torch.zeros(B, 1, H, W, device=dev)
        state = None
        for s in range(L):
            out, state = m(vox[s], prev, state)
            prev = out.clone()
        loss = torch.nn.functional.l1_loss(out, target)
        m.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        if stamped:
            lib.cista_debug_set_fold_stamps(ctypes.c_void_p(buf.data_ptr()), nreg)
        loss.backward()
        torch.cuda.synchronize()
        return lib.cista_debug_set_fold_stamps(None, 0) if stamped else 0

    for _ in range(3):            # warm the clock and the plans
        step(False)
    n = step(True)
    regs = buf.view(nreg, -1).cpu().numpy()
    raw = {}
    for i in range(n):
        st = regs[i].reshape(-1, SLOTS)
        raw[f"launch{i}"] = st[st[:, 1] != 0]
    if os.environ.get("DGRAD_STAMPS_RAW"):
        np.savez_compressed(os.environ["DGRAD_STAMPS_RAW"], **raw)
    for i in range(n):
        s = summarise(regs[i])
        if s:
            print(json.dumps({"launch": i, **s}), flush=True)


if __name__ == "__main__":
    main()
