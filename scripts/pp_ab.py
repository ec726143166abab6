"""Same-process A/B of the two-tile ISTA convs (cista_set_two_tile): per-layer HIP-event times
(bench.time_layers) and the whole-sequence graph replay's frames/s, interleaved passes on one
box, plus bit-identity of the frames of the two arms.
usage: python scripts/pp_ab.py [B] [passes]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402
from v2e2v_amd.sequence import CistaSequence  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 2
H, W, L = 180, 240, 15
dev = torch.device("cuda", 0)
m = CistaLSTCNet([H, W])
bench.he_init_(torch, m, 7)
m = m.to(dev).eval()
vox = bench.synth_voxels(torch, L, B, 5, H, W, 15000, 1000, dev)
lib = _lib.lib()
out = {}
recs = {}
arms = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "3,0").split(",")]
for p in range(passes):
    for arm in arms:
        lib.cista_set_two_tile(arm)
        res = bench.time_layers(torch, m, _lib, vox, B, H, W, dev, 20)
        with torch.no_grad():
            seq = CistaSequence(m, vox)
            seq.run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                r, _ = seq.run()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 3
            recs[arm] = r.clone()
            seq.close()
        key = f"pp{arm}"
        out.setdefault(key, []).append({"fps": round(B * L / dt, 1),
                                        "ista_D": round(res["ista_D"]["ms"], 4),
                                        "ista_P": round(res["ista_P"]["ms"], 4),
                                        "frame_ms": round(sum(v["ms"] * v["launches_per_frame"] for v in res.values()), 3)})
        print(json.dumps({key: out[key][-1]}), flush=True)
out["bit_identical"] = all(bool(torch.equal(recs[arms[0]], recs[a])) for a in arms)
print(json.dumps(out), flush=True)
