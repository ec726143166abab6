"""The bench's voxelizer workload alone (960 windows x 15 000 events -> normalised 5-bin
180x240 voxels), for rocprofv3 kernel statistics of exactly that call size.
usage: rocprofv3 --kernel-trace --stats -- python3 scripts/vox_prof.py [windows] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 960
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
print(json.dumps(bench.time_voxelizer(torch, n, 15000, 5, 180, 240, torch.device("cuda", 0), reps=reps,
                                      cpu_leg=False)))
