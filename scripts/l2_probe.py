"""Diagnostic (GPU): what ISTA P's HBM traffic costs in clock and time.  The same
ISTA P launch at batch B, (a) as built, (b) with its z aux reads and in-place z writes wrapped into
the first 2 MB / 4 MB of z (real, non-zero data that stays L2-resident; the x halo loads are
unchanged), interleaved on one box.  Needs the diagnostic build v2e2v_amd/variants/probe.so
(scripts/build_variants.sh probe "-DCISTA_PROBE=1"); results of the wrapped launches are wrong.
Run it under `rocprofv3 --pmc GRBM_GUI_ACTIVE` to get each kernel's held clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration; the wrapped kernel is conv3x3_split3<..., 13, ...>).
usage: CISTA_HIP_LIB=v2e2v_amd/variants/probe.so python scripts/l2_probe.py [B] [REPS] [OUT]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 100
out = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/l2_probe.json"
H, W = 180, 240
dev = torch.device("cuda", 0)
m = CistaLSTCNet([H, W])
bench.he_init_(torch, m, 7)
m = m.to(dev).eval()
L = _lib.lib()
L.cista_debug_set_ista_p_probe.argtypes = [ctypes.c_uint]
vox = bench.synth_voxels(torch, 2, B, 5, H, W, 15000, 1, dev)
C, h, w = m.base_channels, H // 2, W // 2
lid = _lib.LAYERS.index("ista_P")
with torch.no_grad():
    rec0, st0 = m(vox[0], torch.zeros(B, 1, H, W, device=dev), None)
    cl = torch.channels_last
    outs = [torch.empty(B, 1, H, W, device=dev)] + [
        torch.empty(B, c, h, w, device=dev, memory_format=cl) for c in (2 * C, 2 * C, C, C)]
    ws = m.workspace(B, H, W, dev)
    packed = m.packed_params()
    ev = vox[1].contiguous()
    io = _lib.CistaFrameIO(ev.data_ptr(), rec0.data_ptr(), st0[0].data_ptr(), st0[1].data_ptr(),
                           st0[2][0].data_ptr(), st0[2][1].data_ptr(), *[t.data_ptr() for t in outs])
    cfg = m._cfg()
    stream = torch.cuda.current_stream(dev)
    _lib.check(L.cista_forward(ctypes.byref(cfg), packed.data_ptr(), B, H, W, ctypes.byref(io),
                               ws.data_ptr(), ws.numel(), stream.cuda_stream), "forward")

    def launch():
        _lib.check(L.cista_launch_layer(ctypes.byref(cfg), packed.data_ptr(), lid, B, H, W, ctypes.byref(io),
                                        ws.data_ptr(), ws.numel(), stream.cuda_stream), "ista_P")

    def timed(mask):
        L.cista_debug_set_ista_p_probe(mask)
        for _ in range(3):
            launch()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(REPS):
            launch()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / REPS

    arms = {"as_built": 0, "z_in_2MB": (1 << 19) - 1, "z_in_4MB": (1 << 20) - 1}
    res = {k: [] for k in arms}
    for rep in range(3):                   # interleaved passes
        for k, mask in arms.items():
            res[k].append(round(timed(mask), 4))
    L.cista_debug_set_ista_p_probe(0)
summary = {"B": B, "reps_per_arm_pass": REPS, "ista_P_ms": res,
           "note": "z_in_*: ISTA P with its z aux reads and in-place z writes wrapped into the first "
                   "2 / 4 MB of z (L2-resident real data, results wrong); x halo loads unchanged"}
print(json.dumps(summary))
with open(out, "w") as f:
    json.dump(summary, f, indent=1)
