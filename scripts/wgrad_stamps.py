"""Phase timeline of wgrad_tr_kernel from a CISTA_STAMPS=1 diagnostic build.

usage: CISTA_HIP_LIB=v2e2v_amd/variants/stamps.so python scripts/wgrad_stamps.py [B]

Runs the training step's dominant launch (cista_wgrad_ista_p: the tied ISTA P weight gradient
over depth x B samples at 90 x 120) and reads the per-workgroup timestamps of the MFMA wave and
the staging wave (cista_backward.hpp, WT_STAMP).  Prints, in shader cycles, the median / p90 of:
the MFMA work of one tile, the MFMA wave's wait at the tile barrier, the staging wave's commit
(wait for the tile's loads + fp16 split + LDS stores), its barrier wait, the prologue and the
partial-sum stores, and the in-kernel clock."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402


def q(x):
    x = np.asarray(x, np.int64)
    return (int(np.median(x)), int(np.percentile(x, 90))) if len(x) else None


def analyse(st):
    st = st.reshape(-1, 2, 256).astype(np.int64)
    st = st[st[:, 0, 0] != 0]
    mf, ld = st[:, 0], st[:, 1]
    comp, wait, commit, lwait, issue = [], [], [], [], []
    for m, l in zip(mf, ld):
        n = int(np.sum(m[2:242:2] != 0))
        for it in range(n):
            start = m[1] if it == 0 else m[3 + 2 * (it - 1)]
            comp.append(m[2 + 2 * it] - start)
            wait.append(m[3 + 2 * it] - m[2 + 2 * it])
        for it in range(80):
            a, b, c = l[3 + 3 * it], l[4 + 3 * it], l[5 + 3 * it]
            start = l[2] if it == 0 else l[5 + 3 * (it - 1)]
            if a and start:
                commit.append(a - start)
            if a and b:
                issue.append(b - a)
            if b and c:
                lwait.append(c - b)
    clk = float(np.median((mf[:, 251] - mf[:, 0]) / np.maximum(1, mf[:, 253] - mf[:, 252]) * 100.0))
    return {"workgroups": int(len(st)), "clock_mhz": round(clk),
            "tiles_per_wg": q(np.sum(mf[:, 2:242:2] != 0, axis=1)),
            "mfma_tile": q(comp), "mfma_barrier_wait": q(wait),
            "stage_commit": q(commit), "stage_issue": q(issue), "stage_barrier_wait": q(lwait),
            "prologue": q(mf[:, 1] - mf[:, 0]), "first_commit": q(ld[:, 1] - ld[:, 0]),
            "partials_store": q(mf[:, 251] - mf[:, 250]), "total": q(mf[:, 251] - mf[:, 0])}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    H, W = 180, 240
    dev = torch.device("cuda", 0)
    model = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5).to(dev)
    L = _lib.lib()
    L.cista_debug_set_wstamps.argtypes = [ctypes.c_void_p]
    C, D = model.base_channels, model.depth
    n = D * B * (H // 2) * (W // 2)
    g = torch.Generator(device=dev).manual_seed(11)
    G = (torch.rand(n * 2 * C, device=dev, generator=g) * 2 - 1) * 8192.0
    X = torch.rand(n * C, device=dev, generator=g) * 2 - 1
    sc = torch.tensor([1.0, 1.0], device=dev)
    dW = torch.empty(2 * C * C * 9, device=dev)
    db = torch.empty(2 * C, device=dev)
    ws = model.train_workspace(B, H, W, dev)
    cfg = model._cfg()
    s = torch.cuda.current_stream(dev).cuda_stream
    args = (ctypes.byref(cfg), B, H, W, G.data_ptr(), X.data_ptr(), sc.data_ptr(), dW.data_ptr(), db.data_ptr(),
            ws.data_ptr(), ws.numel(), s)
    buf = torch.zeros(512 * 4096, dtype=torch.int64, device=dev)
    for _ in range(40):          # warm the clock
        _lib.check(L.cista_wgrad_ista_p(*args), "cista_wgrad_ista_p")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        L.cista_wgrad_ista_p(*args)
    e1.record()
    e1.synchronize()
    launch_ms = e0.elapsed_time(e1) / 20
    L.cista_debug_set_wstamps(ctypes.c_void_p(buf.data_ptr()))
    _lib.check(L.cista_wgrad_ista_p(*args), "cista_wgrad_ista_p")
    torch.cuda.synchronize()
    L.cista_debug_set_wstamps(ctypes.c_void_p(0))
    out = analyse(buf.cpu().numpy())
    out["launch_ms_unstamped"] = round(launch_ms, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
