"""Emulator-only timing at config c5's size (bench.py --mode v2e2v settings: 720x1280, 10-frame
packs, V2E2VNet's noise settings): ms per pack over HIP events, for A/B builds and rocprofv3.
usage: python scripts/v2e_prof.py [packs] [height width]"""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from v2e2v_amd.v2e import V2E2VNet  # noqa: E402


def main():
    packs = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    H, W = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (720, 1280)
    P, dt = 10, 1.0 / 240.0
    dev = torch.device("cuda", 0)
    cfgs = types.SimpleNamespace(event_mode="voxel_grid", num_bins=5, pl=1.0, ps=1.0, ql=1.0, qs=1.0, C=0.2,
                                 threshold_sigma=0.03, cutoff_hz=30.0, refractory_period_s=0.001,
                                 base_channels=64, depth=5)
    net = V2E2VNet(cfgs, [H, W], dev, lazy_count=True)
    yy, xx = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    n_frames = packs * (P - 1) + 1
    vid = torch.empty(n_frames, 1, H, W, device=dev)
    for f in range(n_frames):
        bg = 60 + 40 * torch.sin((xx + 2.0 * f) / 23.0) * torch.cos(yy / 31.0)
        blob = 170 * torch.exp(-((xx - 100 - 6.0 * f) ** 2 + (yy - H / 2) ** 2) / 800.0)
        vid[f, 0] = (bg + blob).clamp(0, 255)
    emu = net.v2e_net
    with torch.no_grad():
        def run():
            emu.reset()
            for k in range(packs):
                fr = vid[k * (P - 1): k * (P - 1) + P].permute(1, 0, 2, 3).contiguous()
                ts = ((k * (P - 1)) * dt + dt * torch.arange(P, dtype=torch.float64)).repeat(1, 1)
                emu(fr, ts)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        e1.synchronize()
    print(f"emulator {H}x{W}: {e0.elapsed_time(e1) / packs:.4f} ms per {P}-frame pack, "
          f"events last pack {int(emu.num_events) if hasattr(emu, 'num_events') else -1}", flush=True)


if __name__ == "__main__":
    main()
