"""The training step's dominant launch alone (cista_wgrad_ista_p at the bench shapes), for
rocprofv3 PMC passes: python scripts/train_wgrad_bench.py [reps]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet, _lib  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    model = CistaLSTCNet([180, 240], base_channels=64, depth=5, num_bins=5).to(dev)
    r = bench.train_roofline(torch, model, _lib, 8, 180, 240, dev, reps=reps)
    print(r["launch_ms"], r["achieved"], r["frac"])
