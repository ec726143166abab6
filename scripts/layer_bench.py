"""Per-layer kernel timing of one libcista_hip.so build (A/B of tiling variants).
usage: CISTA_HIP_LIB=path python scripts/layer_bench.py [B [H W]]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H, W = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (180, 240)
dev = torch.device("cuda", 0)
m = CistaLSTCNet([H, W])
bench.he_init_(torch, m, 7)
m = m.to(dev).eval()
vox = bench.synth_voxels(torch, 2, B, 5, H, W, 15000, 1, dev)
res = bench.time_layers(torch, m, _lib, vox, B, H, W, dev, 20)
tot = sum(v["ms"] * v["launches_per_frame"] for v in res.values())
print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "B": B, "frame_ms": round(tot, 3),
                  "fps": round(B / tot * 1e3, 1),
                  "ms": {k: round(v["ms"], 4) for k, v in res.items()},
                  "tflops": {k: round(v["tflops"], 1) for k, v in res.items()}}))
