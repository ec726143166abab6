"""Diagnostic (GPU): is a conv layer bound by the energy of its MFMA operands (the chip lowering
its clock under load, MI355X_MICROARCH.md 'DVFS give-back') or by its schedule?  Per-layer HIP-event
times at batch B of the same build, same buffers, with (a) the He-init weights, (b) every weight
zero (the MFMA B operands 0, the same instruction stream, the same HBM / LDS traffic).  A layer
that runs much faster in (b) is held down by its clock, not by its instruction stream.
usage: python scripts/power_probe.py [B] [OUT]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/power_probe.json"
H, W = 180, 240
dev = torch.device("cuda", 0)
m = CistaLSTCNet([H, W])
bench.he_init_(torch, m, 7)
m = m.to(dev).eval()
vox = bench.synth_voxels(torch, 2, B, 5, H, W, 15000, 1, dev)
res = {}
for rep in range(2):                       # two passes: the first warms the clock governor
    res[f"he_{rep}"] = bench.time_layers(torch, m, _lib, vox, B, H, W, dev, 20)
    with torch.no_grad():
        saved = {k: v.clone() for k, v in m.state_dict().items()}
        for k, v in m.state_dict().items():
            if k.endswith("weight"):
                v.zero_()
    m.invalidate_packed()
    res[f"zero_w_{rep}"] = bench.time_layers(torch, m, _lib, vox, B, H, W, dev, 20)
    m.load_state_dict(saved)
summary = {k: {n: round(v["ms"], 4) for n, v in r.items()} for k, r in res.items()}
print(json.dumps(summary))
with open(out, "w") as f:
    json.dump(summary, f, indent=1)
