"""Is the BPTT step host-bound?  Host time to issue the forward / backward / Adam of one step
against the device time of the same step (HIP events): when issuing takes as long as running,
the GPU waits on the launches.  Same workload as `bench.py --mode train` (180x240, len 15, B=8).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from v2e2v_amd import CistaLSTCNet
from v2e2v_amd.losses import SSIM


def main():
    dev = torch.device("cuda:0")
    B, L, H, W, nb = 8, 15, 180, 240, 5
    model = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=nb)
    bench.he_init_(torch, model, seed=7)
    model = model.to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    ssim_fn = SSIM(data_range=1, size_average=True, channel=1, nonnegative_ssim=False)
    vox = bench.synth_voxels(torch, L, B, nb, H, W, 15000, seed=2000, device=dev)
    target = torch.rand(B, 1, H, W, device=dev)
    res = []
    for rep in range(4):
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t0 = time.perf_counter()
        e[0].record()
        prev = torch.zeros(B, 1, H, W, device=dev)
        state = None
        for s in range(L):
            out, state = model(vox[s], prev, state)
            prev = out.clone()
        loss = torch.nn.functional.l1_loss(out, target) + (1 - ssim_fn(out, target))
        e[1].record()
        t1 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        e[2].record()
        t2 = time.perf_counter()
        opt.step()
        e[3].record()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        res.append({"host_issue_ms": {"forward": (t1 - t0) * 1e3, "backward": (t2 - t1) * 1e3, "adam": (t3 - t2) * 1e3},
                    "device_ms": {"forward": e[0].elapsed_time(e[1]), "backward": e[1].elapsed_time(e[2]),
                                  "adam": e[2].elapsed_time(e[3])},
                    "wall_ms": (t4 - t0) * 1e3, "drain_after_issue_ms": (t4 - t3) * 1e3})
    print(json.dumps(res[1:], indent=1))


if __name__ == "__main__":
    main()
