#!/usr/bin/env python3
"""bench.py -- CISTA-LSTC inference throughput on MI355X (BASELINE.json config c2).

Metric: reconstructed frames/s at 180x240, 5-bin voxels, depth 5, base_channels 64.
One STEP = one len_sequence (15) recurrent pass over B sequences per GPU: states carried
frame to frame, prev_image = previous output (reference test_e2v.py:105-117 semantics),
starting from prev_states=None / zero image.  Inputs (synthetic voxels, built on the GPU from
15 000 random events each by the HIP voxelizer, reference utils/event_process.py) are resident
in HBM before the timed region; the voxelizer itself is timed separately ("voxelizer").  value = frames of ALL ranks / max-over-ranks wall time of K steps.

Multi-GPU: one process per GPU (torchrun), sequences sharded across ranks with no data-path
collective (inference replicas: "scaling": "weak"); only the timing max and a barrier use RCCL.

Also reported on the same JSON line:
  roofline      -- the dominant kernel's achieved algorithmic TFLOP/s (HIP events on the stream
                   it is launched on) against the fp16-MFMA dense peak divided by the 3 passes
                   of the split-fp16 scheme;
  cpu_baseline  -- rank 0 only: the reference's forward restated op for op on ATen's CPU kernels
                   (oracle/cista_oracle_torch.py, "kind": "port") timed on this host's cores over
                   a bounded sample (~10 s), and the PSNR / max relative error of the GPU frames
                   against it on the same inputs ("PSNR vs ref" of the metric).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import re
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_F16_MFMA_TFLOPS = 2500.0                # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
SPLIT_PASSES = 3
PEAK_F32_MFMA_TFLOPS = 157.3                 # MI355X dense fp32 matrix (BASELINE.md framing)
HBM_TBPS = 8.0                               # MI355X HBM3E


def parse():
    """Flags: the driver's (--gpus/--steps/--warmup) and the reference harness's names for the
    model / data (utils/configs.py:6-91: --image_dim, -b/--num_bins, -d/--depth,
    -c/--base_channels, -s/--len_sequence, --batch_size, --num_events, --num_pack_frames);
    the older spellings stay as aliases."""
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (= ranks) to measure; without a rank launcher, N > 1 starts N child ranks "
                        "itself (launch_ranks); under torchrun it must equal WORLD_SIZE (default: "
                        "WORLD_SIZE, else 1)")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check without a GPU: the ranks come up over gloo, time a trivial CPU "
                        "step and rank 0 prints the JSON line (n_gpus, ranks_seen); no HIP call")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    # 256 sequences x 15 frames of 180x240 state and voxels are ~4 GB of the 288 GB HBM; the tiles
    # of the last dispatch round are then a smaller share than at 64 (sweep: 7918 / 8061 / 8143 /
    # 8147 frames/s at B = 64 / 128 / 256 / 512)
    p.add_argument("--batch_size", "--batch", dest="batch", type=int, default=256, help="sequences per GPU")
    p.add_argument("-s", "--len_sequence", "--len-seq", dest="len_seq", type=int, default=15)
    p.add_argument("--image_dim", nargs=2, type=int, default=None, metavar=("H", "W"),
                   help="frame height and width (default 180 240; v2e2v mode 720 1280)")
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--width", type=int, default=None)
    p.add_argument("-b", "--num_bins", type=int, default=5)
    p.add_argument("-d", "--depth", type=int, default=5)
    p.add_argument("-c", "--base_channels", type=int, default=64)
    p.add_argument("--num_events", "--num-events", dest="num_events", type=int, default=15000)
    p.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                   help="timed region: the whole L-frame recurrence replayed as one hipGraph "
                        "(v2e2v_amd/sequence.py) or the eager per-frame module calls; auto = both "
                        "measured, the graph replay reported as the headline (fixed, not the "
                        "faster of two noisy timings), the eager time beside it in "
                        "'eager_vs_graph'")
    p.add_argument("--sweep", default="1,8,32,64,128",
                   help="batch sizes of the small-batch / latency sweep (empty: skip)")
    p.add_argument("--cpu-frames", type=int, default=15,
                   help="recurrent frames per CPU-baseline sequence (B=1); sequences repeat to ~10 s")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--layer-reps", type=int, default=10)
    p.add_argument("--adam", choices=["fused", "foreach"], default="fused",
                   help="--mode train: torch.optim.Adam implementation (the same update; fused = one "
                        "multi-tensor kernel per step instead of a chain of foreach launches)")
    p.add_argument("--mode", choices=["infer", "train", "v2e2v"], default="infer",
                   help="infer: the headline metric (config c2); train: BPTT step (configs c3/c4); "
                        "v2e2v: emulator + reconstruction at 720x1280 (config c5)")
    p.add_argument("--num_pack_frames", "--pack-frames", dest="pack_frames", type=int, default=10,
                   help="v2e2v: frames per reconstruction")
    args = p.parse_args()
    given = lambda *names: any(a in sys.argv for a in names)    # noqa: E731
    if args.mode == "train" and not given("--batch", "--batch_size"):
        args.batch = 8            # BASELINE config c3: batch 8 per GPU (c4: 8 GPUs x 8 = 64)
    H, W = (180, 240) if args.mode != "v2e2v" else (720, 1280)
    if args.image_dim:
        H, W = args.image_dim
    args.height = args.height or H
    args.width = args.width or W
    if args.mode == "v2e2v" and not given("--batch", "--batch_size"):
        args.batch = 1            # config c5: one HFR video per GPU
    return args


def v2e2v_main(args, torch, vd, rank, world, device):
    """Config c5 (model_v2e2v.py:72-128, test.py): per step, len_sequence reconstructions, each
    from num_pack_frames high-frame-rate frames -> EventEmulator (voxel grid, V2E2VNet's noise
    settings) -> CistaLSTCNet, states and prev image carried.  Replicas per GPU (independent
    videos), frames/s = reconstructions of all ranks / max-over-ranks time."""
    import types
    from v2e2v_amd.v2e import V2E2VNet
    B, L, H, W, P = args.batch, args.len_seq, args.height, args.width, args.pack_frames
    cfgs = types.SimpleNamespace(event_mode="voxel_grid", num_bins=args.num_bins, pl=1.0, ps=1.0, ql=1.0, qs=1.0,
                                 C=0.2, threshold_sigma=0.03, cutoff_hz=30.0, refractory_period_s=0.001,
                                 base_channels=args.base_channels, depth=args.depth)
    net = V2E2VNet(cfgs, [H, W], device, lazy_count=True)    # no host sync per pack
    he_init_(torch, net.e2v_net, seed=7)
    net = net.to(device).eval()
    # synthetic HFR video resident in HBM: a textured background panning + a moving bright blob
    g = torch.Generator(device=device).manual_seed(100 + rank)
    yy, xx = torch.meshgrid(torch.arange(H, device=device, dtype=torch.float32),
                            torch.arange(W, device=device, dtype=torch.float32), indexing="ij")
    noise = torch.rand(B, 1, H, W, generator=g, device=device) * 4
    n_frames = L * (P - 1) + 1
    vid = torch.empty(n_frames, B, H, W, device=device)
    for f in range(n_frames):
        bg = 60 + 40 * torch.sin((xx + 2.0 * f) / 23.0) * torch.cos(yy / 31.0)
        blob = 170 * torch.exp(-((xx - 100 - 6.0 * f) ** 2 + (yy - H / 2) ** 2) / 800.0)
        vid[f] = (bg + blob + noise[:, 0]).clamp(0, 255)
    dt = 1.0 / 240.0

    def step(seq):
        pred, states = None, None
        for k in range(L):
            frames = vid[k * (P - 1): k * (P - 1) + P].permute(1, 0, 2, 3).contiguous()
            t0 = (seq * n_frames + k * (P - 1)) * dt
            ts = (t0 + dt * torch.arange(P, dtype=torch.float64)).repeat(B, 1)
            pred, states = net(frames, ts, pred, states, seq_idx=seq)
        return pred

    with torch.no_grad():
        seq = 0
        for _ in range(args.warmup):
            step(seq)
            seq += 1
        torch.cuda.synchronize()
        vd.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            rec = step(seq)
            seq += 1
        torch.cuda.synchronize()
        vd.barrier()
        elapsed = vd.max_over_ranks(time.perf_counter() - t0, device)
    frames_done = world * B * L * args.steps
    from v2e2v_amd import _lib
    # the dominant kernel of the reconstruction at this size (HIP events on the library's stream)
    vlast = net.event_voxel_grids
    layers = time_layers(torch, net.e2v_net, _lib, torch.stack([vlast, vlast]), B, H, W, device, args.layer_reps)
    roofline = dominant_roofline(layers, _lib, traffic_tag="v2e2v")
    # the emulator alone: one pack of P frames (diff / iters / emit per frame + preprocess)
    with torch.no_grad():
        frames = vid[:P].permute(1, 0, 2, 3).contiguous()
        net.v2e_net.reset()
        ts0 = (dt * torch.arange(P, dtype=torch.float64)).repeat(B, 1)
        net.v2e_net(frames, ts0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for r in range(reps):
            net.v2e_net(frames, ts0 + (r + 1) * P * dt)
        e1.record()
        e1.synchronize()
        v2e_ms = e0.elapsed_time(e1) / reps
        # output_mode='raw' on the same packs: count pass + row pass, one host sync per call
        from v2e2v_amd.v2e import EventEmulator
        raw = EventEmulator("raw", num_bins=cfgs.num_bins, pos_thres=cfgs.C, neg_thres=cfgs.C,
                            sigma_thres=cfgs.threshold_sigma, cutoff_hz=cfgs.cutoff_hz,
                            refractory_period_s=cfgs.refractory_period_s, leak_rate_hz=0.1, shot_noise_rate_hz=1,
                            device=device, seed=5)
        raw(frames, ts0)
        t_raw = time.perf_counter()
        raw_events = 0
        for r in range(reps):
            raw_events += raw(frames, ts0 + (r + 1) * P * dt)[1]
        torch.cuda.synchronize()
        raw_ms = (time.perf_counter() - t_raw) * 1e3 / reps
    cpu = None
    if world == 1 and not args.no_cpu_baseline:       # the CPU leg: rank 0 at N=1 only
        cpu = v2e2v_cpu_baseline(torch, net, vid, cfgs, B, H, W, P, dt)
    if rank == 0:
        print(json.dumps({
            "metric": "V2E2V reconstructed frames/sec (v2e emulator + CISTA-LSTC) at 720x1280",
            "value": round(frames_done / elapsed, 2), "unit": "frames/s", "n_gpus": world, **pg_info(vd),
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic HFR video (panning texture + moving blob), random-init weights",
            "config": {"workload": f"V2E2V {H}x{W}, num_pack_frames={P}, len_sequence={L}, {B} video/GPU",
                       "batch_per_gpu": B, "len_sequence": L, "num_pack_frames": P,
                       "parallelism": f"replicas x{world}"},
            "events_last_pack": int(net.num_events), "outputs_finite": bool(torch.isfinite(rec).all()),
            "roofline": roofline, "cpu_baseline": cpu,
            "emulator_ms_per_pack": round(v2e_ms, 4),
            "emulator_raw_mode": {"ms_per_pack": round(raw_ms, 4), "events_per_pack": raw_events // reps,
                                  "events_per_s": round(raw_events / (raw_ms * reps / 1e3), 1)},
            "reconstruction_ms_per_frame_kernels": round(sum(v["ms"] * v["launches_per_frame"]
                                                             for v in layers.values()), 4),
            "layers_ms": {k: round(v["ms"], 4) for k, v in layers.items()}}),
            flush=True)
    vd.finalize()


class _NpRng:
    """The random source the emulator restatement draws from (numpy; the GPU emulator's Philox
    stream is not reproduced -- the CPU leg is a timing sample, not a parity check)."""

    def __init__(self, seed):
        import numpy as np
        self.g = np.random.default_rng(seed)

    def normal(self, mean, std, shape):
        return self.g.normal(mean, std, shape)

    def randn(self, shape):
        return self.g.standard_normal(shape, dtype="float32")

    def rand(self, shape):
        return self.g.random(shape, dtype="float32")


def v2e2v_cpu_baseline(torch, net, vid, cfgs, B, H, W, P, dt, min_s=10.0, max_recs=6):
    """cpu_baseline leg of config c5: the emulator restated in numpy (oracle/v2e_oracle.py:
    EventEmulator voxel-grid mode, the V2E2VNet noise settings) + event_preprocess + the
    CISTA-LSTC forward on ATen's CPU kernels (oracle/cista_oracle_torch.py), B=1, reconstruction
    after reconstruction (states and previous image carried) until >= min_s seconds."""
    import numpy as np
    from oracle import fixtures as fx
    from oracle import v2e_oracle as vo
    from oracle.cista_oracle_torch import CistaLSTCTorchCPU
    cores, core_note = host_cores()
    torch.set_num_threads(cores)
    e2v = net.e2v_net
    sd = {k: v.detach().cpu().numpy() for k, v in e2v.state_dict().items()}
    ref = CistaLSTCTorchCPU(fx.collapse_tied(sd, e2v.depth), e2v.depth)
    emu = vo.V2EOracle(num_bins=cfgs.num_bins, pos_thres=cfgs.C, neg_thres=cfgs.C, sigma_thres=cfgs.threshold_sigma,
                       cutoff_hz=cfgs.cutoff_hz, refractory_period_s=cfgs.refractory_period_s, leak_rate_hz=0.1,
                       shot_noise_rate_hz=1.0, rng=_NpRng(0))
    n_avail = (vid.shape[0] - 1) // (P - 1)
    prev, states, recs, t = torch.zeros(1, 1, H, W), None, 0, 0.0
    while recs < min(max_recs, n_avail) and (t < min_s or recs == 0):
        fr = vid[recs * (P - 1): recs * (P - 1) + P, :1].permute(1, 0, 2, 3).cpu().numpy()
        ts = (recs * (P - 1) + np.arange(P)[None]) * dt
        t0 = time.perf_counter()
        vox, _ = emu.forward(fr, ts)
        v = torch.from_numpy(np.ascontiguousarray(vo.preprocess_whole(vox)))
        prev, states = ref.forward(v, prev, states)
        t += time.perf_counter() - t0
        recs += 1
    return dict(value=recs / t, unit="frames/s", cores=int(cores), kind="port",
                sample=f"{recs} reconstruction(s) at {H}x{W} (B=1), each a {P}-frame pack through the numpy "
                       f"emulator restatement (oracle/v2e_oracle.py) + the PyTorch-CPU CISTA-LSTC restatement "
                       f"(oracle/cista_oracle_torch.py), {core_note}, {t:.1f} s")


def train_main(args, torch, vd, rank, world, device):
    """BPTT training step of train_e2v.py:108-130 on the HIP path: len_sequence frames with
    prev_img = output.clone() (no detach) and states carried, loss on the last frame, one
    backward through the whole sequence, Adam step.  Loss = L1 + (1 - SSIM) as train_e2v.py:
    117-120 (SSIM on the HIP path, v2e2v_amd/losses.py); the reference also adds LPIPS-VGG, whose
    weights need a network download.  Multi-GPU: DistributedDataParallel over RCCL
    (one gradient all-reduce per step)."""
    from v2e2v_amd import CistaLSTCNet
    from v2e2v_amd.losses import SSIM
    ssim_fn = SSIM(data_range=1, size_average=True, channel=1, nonnegative_ssim=False)
    B, L, H, W = args.batch, args.len_seq, args.height, args.width
    nb, C, depth = args.num_bins, args.base_channels, args.depth
    model = CistaLSTCNet([H, W], base_channels=C, depth=depth, num_bins=nb)
    he_init_(torch, model, seed=7)
    model = model.to(device).train()
    net = model
    if vd.active():
        # under torchrun (any N, N=1 included): one bucketed RCCL all-reduce of the gradients
        net = torch.nn.parallel.DistributedDataParallel(model, device_ids=[device.index],
                                                        broadcast_buffers=False)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, **({"fused": True} if args.adam == "fused" else {}))
    vox = synth_voxels(torch, L, B, nb, H, W, args.num_events, seed=2000 + rank, device=device)
    target = torch.rand(B, 1, H, W, device=device, generator=torch.Generator(device=device).manual_seed(3))

    def step():
        prev = torch.zeros(B, 1, H, W, device=device)
        state = None
        for s in range(L):
            out, state = net(vox[s], prev, state)
            prev = out.clone()
        loss = torch.nn.functional.l1_loss(out, target) + (1 - ssim_fn(out, target))
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    vd.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    vd.barrier()
    elapsed = vd.max_over_ranks(time.perf_counter() - t0, device)
    frames = world * B * L * args.steps
    from v2e2v_amd import _lib
    macs_frame, _ = frame_work(_lib, model, H, W)
    # a BPTT frame costs the forward plus dgrad and wgrad of every conv: 3x the forward FLOPs
    # (SURVEY 8(d) "training FLOPs ~ 3x fwd"), run on the same split-f16 MFMA peak
    train_tf = frames / elapsed / world * 3 * 2 * macs_frame / 1e12
    peak = PEAK_F16_MFMA_TFLOPS / SPLIT_PASSES
    roofline = train_roofline(torch, model, _lib, B, H, W, device)
    roofline["step_tflops_est"] = round(train_tf, 2)
    roofline["step_frac_est"] = round(train_tf / peak, 4)
    roofline["step_note"] = "whole BPTT step: 3 x forward algorithmic FLOPs per frame x frames/s per GPU"
    cpu = None
    if world == 1 and not args.no_cpu_baseline:       # the CPU leg: rank 0 at N=1 only
        cpu = train_cpu_baseline(torch, model, vox, target, L, H, W)
    if rank == 0:
        print(json.dumps({
            "metric": "BPTT training frames/sec at 180x240 5-bin depth=5 (len_sequence 15)",
            "value": round(frames / elapsed, 2), "unit": "frames/s", "n_gpus": world, **pg_info(vd),
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (GPU-generated 15000-event voxels, random targets; L1 + 1-SSIM loss)",
            "config": {"workload": f"train_e2v BPTT len {L}, batch {B}/GPU, {H}x{W}",
                       "batch_per_gpu": B, "global_batch": B * world, "len_sequence": L,
                       "parallelism": f"ddp{world}" if vd.active() else "single",
                       "process_group": (torch.distributed.get_backend() if vd.active() else None),
                       "optimizer": f"torch.optim.Adam lr 1e-4 ({args.adam})"},
            "loss": float(loss.item()),
            "roofline": roofline, "cpu_baseline": cpu,
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 2)}), flush=True)
    vd.finalize()


def train_roofline(torch, model, lib_mod, B, H, W, device, reps=10):
    """The training step's dominant kernel: the tied ISTA P weight gradient over all depth
    iterations (split-f16 wgrad_tr_kernel + its partial reduction, cista_wgrad_ista_p), timed
    alone with HIP events on the stream it is launched on, at the bench's shapes (synthetic G / X
    of the same sizes; the work does not depend on the values).  Algorithmic FLOPs per launch =
    2 x 9 x 2C x C x (depth x B x h x w); HBM bytes per launch from the committed PMC passes of
    this build (profiles/rNN_train_pmc_traffic.json, scripts/pmc_train_wgrad.sh)."""
    L = lib_mod.lib()
    C, D = model.base_channels, model.depth
    h, w = H // 2, W // 2
    n = D * B * h * w
    g = torch.Generator(device=device).manual_seed(11)
    G = (torch.rand(n * 2 * C, device=device, generator=g) * 2 - 1) * 8192.0    # split scale folded in
    X = torch.rand(n * C, device=device, generator=g) * 2 - 1
    sc = torch.tensor([1.0, 1.0], device=device)
    dW = torch.empty(2 * C * C * 9, device=device)
    db = torch.empty(2 * C, device=device)
    ws = model.train_workspace(B, H, W, device)
    cfg = model._cfg()
    stream = torch.cuda.current_stream(device)
    args = (ctypes.byref(cfg), B, H, W, G.data_ptr(), X.data_ptr(), sc.data_ptr(), dW.data_ptr(), db.data_ptr(),
            ws.data_ptr(), ws.numel(), stream.cuda_stream)
    for _ in range(2):
        lib_mod.check(L.cista_wgrad_ista_p(*args), "cista_wgrad_ista_p")
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        L.cista_wgrad_ista_p(*args)
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flop = 2.0 * 9 * 2 * C * C * n
    tf = flop / (ms * 1e-3) / 1e12
    peak = PEAK_F16_MFMA_TFLOPS / SPLIT_PASSES
    alg = 4.0 * n * 3 * C                     # G (2C) and X (C) read once, fp32
    roof = dict(bound="mfma", achieved=round(tf, 2), peak=round(peak, 1), unit="TFLOP/s",
                frac=round(tf / peak, 4), traffic=None,
                kernel="ista_P_wgrad (wgrad_tr_kernel + reduce_partials_kernel, all %d iterations)" % D,
                launch_ms=round(ms, 4), flop_per_launch=flop, algorithmic_bytes_per_launch=alg,
                note="achieved = algorithmic fp32 FLOPs (2 x MACs) of one launch / its mean duration "
                     "(HIP events); peak = 2500 TFLOP/s dense fp16 MFMA / 3 split passes")
    import glob
    import hashlib
    tfiles = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_train_pmc_traffic.json"))
                    if re.fullmatch(r"r\d\d_train_pmc_traffic\.json", os.path.basename(f)))
    if tfiles:
        try:
            tj = json.load(open(tfiles[-1]))
            roof["traffic_source"] = os.path.relpath(tfiles[-1], ROOT)
            tl = tj["layers"].get("ista_P_wgrad")
            if tl and tj.get("lib_sha256") == hashlib.sha256(open(lib_mod.LIB_PATH, "rb").read()).hexdigest():
                roof["traffic"] = tl["hbm_bytes_per_launch"]
                gbps = tl["hbm_bytes_per_launch"] / (ms * 1e-3) / 1e9
                roof["hbm_achieved_GBps"] = round(gbps, 1)
                roof["hbm_frac"] = round(gbps / (HBM_TBPS * 1e3), 4)
            else:
                roof["traffic_note"] = "no PMC traffic of this build in " + roof["traffic_source"]
        except (OSError, ValueError, KeyError):
            pass
    return roof


def train_cpu_baseline(torch, model, vox, target, L, H, W, min_s=10.0, max_steps=4):
    """The training step's CPU baseline: the PyTorch-CPU restatement (oracle/cista_oracle_torch.py,
    pinned to the golden vectors) under autograd -- train_e2v.py:108-130 semantics, B=1, the
    same L frames and size -- on this host's cores, repeated to ~10 s."""
    from oracle import fixtures as fx
    from oracle.cista_oracle_torch import CistaLSTCTorchCPU, bptt_step
    cores, core_note = host_cores()
    torch.set_num_threads(cores)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    net = CistaLSTCTorchCPU(fx.collapse_tied(sd, model.depth), model.depth, requires_grad=True)
    v = vox[:, :1].cpu().numpy()
    tg = target[:1].cpu().numpy()
    steps, dt = 0, 0.0
    while steps < max_steps and (dt < min_s or steps == 0):
        t0 = time.perf_counter()
        bptt_step(net, v, tg)
        dt += time.perf_counter() - t0
        steps += 1
    return dict(value=steps * L / dt, unit="frames/s", cores=int(cores), kind="port",
                sample=f"{steps} BPTT step(s) of {L} frames at {H}x{W}, B=1 (L1 on the last frame, "
                       f"autograd through the PyTorch-CPU restatement), {core_note}, {dt:.1f} s")


# ------------------------------------------------------------------ synthetic inputs (GPU)
def synth_events(torch, n_windows, n_events, H, W, seed, device):
    """n_windows windows of n_events events each, concatenated: (N, 4) float64 rows (t, x, y, p)
    with sorted t ~ U(0, 0.05), x, y uniform, p in {0, 1} (SURVEY 8(c)(ii) recipe), generated on
    the device; offsets (n_windows + 1,) int64."""
    g = torch.Generator(device=device).manual_seed(seed)
    t = torch.sort(torch.rand(n_windows, n_events, generator=g, device=device, dtype=torch.float64) * 0.05, 1)[0]
    x = torch.randint(0, W, (n_windows, n_events), generator=g, device=device).to(torch.float64)
    y = torch.randint(0, H, (n_windows, n_events), generator=g, device=device).to(torch.float64)
    p = torch.randint(0, 2, (n_windows, n_events), generator=g, device=device).to(torch.float64)
    ev = torch.stack([t, x, y, p], -1).view(-1, 4).contiguous()
    off = torch.arange(0, n_windows * n_events + 1, n_events, dtype=torch.int64, device=device)
    return ev, off


def synth_voxels(torch, n_frames, n_seq, nb, H, W, n_events, seed, device):
    """(n_frames, n_seq, nb, H, W) fp32 voxels from synthetic events through the HIP voxelizer
    (events_to_voxel_grid + event_preprocess(filter_hot_pixel=True), reference
    utils/event_process.py:15-63,132-154)."""
    from v2e2v_amd import event_process as ep
    ev, off = synth_events(torch, n_frames * n_seq, n_events, H, W, seed, device)
    vox = ep.events_to_voxel_batch((ev, off), nb, W, H, mode="std", filter_hot_pixel=True, device=device)
    return vox.view(n_frames, n_seq, nb, H, W)


def time_voxelizer(torch, n_windows, n_events, nb, H, W, device, reps=5, cpu_leg=True):
    """SURVEY 8 row f1, timed separately from the metric: events resident in HBM -> normalised
    voxels, n_windows windows per call (HIP events on the current stream)."""
    from v2e2v_amd import event_process as ep
    ev, off = synth_events(torch, n_windows, n_events, H, W, 99, device)
    out = torch.empty(n_windows, nb, H, W, device=device)
    ep.events_to_voxel_batch((ev, off), nb, W, H, mode="std", filter_hot_pixel=True, out=out, device=device,
                             strict=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ep.events_to_voxel_batch((ev, off), nb, W, H, mode="std", filter_hot_pixel=True, out=out, device=device,
                                 strict=False)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    res = {"windows_per_call": n_windows, "events_per_window": n_events, "ms_per_call": round(ms, 3),
           "windows_per_s": round(n_windows / ms * 1e3, 1),
           "events_per_s": round(n_windows * n_events / ms * 1e3, 1)}
    if cpu_leg:
        # cpu_baseline leg of the voxelizer: the numpy restatement of the reference path (oracle/,
        # bit-identical to the GPU result), 4 windows on 1 host core; also checks the GPU output
        from oracle import fixtures as fx
        evs = ev[: 4 * n_events].cpu().numpy().reshape(4, n_events, 4)
        t0 = time.perf_counter()
        ref = [fx.normalize_voxel(fx.voxelize(w, nb, W, H), True) for w in evs]
        cpu_ms = (time.perf_counter() - t0) / len(evs) * 1e3
        got = out[:4].cpu().numpy()
        res["cpu_baseline"] = {"value": round(1e3 / cpu_ms, 1), "unit": "windows/s", "cores": 1, "kind": "port",
                               "sample": "4 windows of the same workload (numpy restatement)"}
        res["bit_exact_vs_ref"] = bool(all((g == r).all() for g, r in zip(got, ref)))
    return res


def he_init_(torch, model, seed):
    """Random-init weights of the architecture, He-scaled so that the recurrence is not
    trivially saturated (the default init gives ~0.5 everywhere)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, prm in model.named_parameters():
            if name.endswith("Lambda"):
                prm.fill_(0.05)
            elif prm.dim() == 4:
                fan_in = prm.shape[1] * 9
                prm.copy_(torch.randn(prm.shape, generator=g) / math.sqrt(fan_in))
            else:
                prm.copy_(torch.rand(prm.shape, generator=g) * 0.2 - 0.1)


def run_sequence(torch, model, vox_seq, B, H, W, device):
    prev = torch.zeros(B, 1, H, W, device=device)
    states = None
    for f in range(vox_seq.shape[0]):
        prev, states = model(vox_seq[f], prev, states)
    return prev, states


def time_layers(torch, model, lib_mod, vox, B, H, W, device, reps):
    """Average duration of every kernel of the frame schedule, measured with HIP events on the
    stream the library launches on (torch's current stream, passed explicitly)."""
    L = lib_mod.lib()
    C = model.base_channels
    h, w = H // 2, W // 2
    with torch.no_grad():
        rec0, st0 = model(vox[0], torch.zeros(B, 1, H, W, device=device), None)
        cl = torch.channels_last
        outs = dict(rec=torch.empty(B, 1, H, W, device=device),
                    c_lstc=torch.empty(B, 2 * C, h, w, device=device, memory_format=cl),
                    z=torch.empty(B, 2 * C, h, w, device=device, memory_format=cl),
                    h=torch.empty(B, C, h, w, device=device, memory_format=cl),
                    c=torch.empty(B, C, h, w, device=device, memory_format=cl))
        ws = model.workspace(B, H, W, device)
        packed = model.packed_params()
        ev = vox[1].contiguous()
        io = lib_mod.CistaFrameIO(ev.data_ptr(), rec0.data_ptr(), st0[0].data_ptr(),
                                  st0[1].data_ptr(), st0[2][0].data_ptr(), st0[2][1].data_ptr(),
                                  outs["rec"].data_ptr(), outs["c_lstc"].data_ptr(),
                                  outs["z"].data_ptr(), outs["h"].data_ptr(), outs["c"].data_ptr())
        cfg = model._cfg()
        stream = torch.cuda.current_stream(device)
        lib_mod.check(L.cista_forward(ctypes.byref(cfg), packed.data_ptr(), B, H, W, ctypes.byref(io),
                                      ws.data_ptr(), ws.numel(), stream.cuda_stream), "forward")
        res = {}
        for lid, name in enumerate(lib_mod.LAYERS):
            for _ in range(2):
                lib_mod.check(L.cista_launch_layer(ctypes.byref(cfg), packed.data_ptr(), lid, B, H, W,
                                                   ctypes.byref(io), ws.data_ptr(), ws.numel(),
                                                   stream.cuda_stream), name)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                L.cista_launch_layer(ctypes.byref(cfg), packed.data_ptr(), lid, B, H, W,
                                     ctypes.byref(io), ws.data_ptr(), ws.numel(), stream.cuda_stream)
            e1.record(stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / reps
            macs = L.cista_layer_macs(ctypes.byref(cfg), lid, B, H, W)
            per_frame = model.depth if name in ("ista_D", "ista_P") else 1
            res[name] = dict(ms=ms, macs=macs, launches_per_frame=per_frame,
                             tflops=2 * macs / (ms * 1e-3) / 1e12)
        torch.cuda.synchronize()
    # the input stage computes W0 too (one composed linear map, input_w0_kernel): the W0 layer
    # launches nothing (the build says so), so its work is credited to the fused launch
    cfg = model._cfg()
    if "W0" in res and L.cista_layer_fused(ctypes.byref(cfg), lib_mod.LAYERS.index("W0")):
        w0 = res.pop("W0")
        res["input+W0"] = dict(res.pop("input"))
        r = res["input+W0"]
        r["macs"] += w0["macs"]
        r["tflops"] = 2 * r["macs"] / (r["ms"] * 1e-3) / 1e12
    return res


def dominant_roofline(layers, lib_mod, traffic_tag=None):
    """The roofline object of the frame's dominant kernel (largest ms x launches per frame):
    algorithmic FLOPs of one launch / its mean duration (HIP events, time_layers), against the
    split3 peak; HBM bytes per launch from the committed PMC passes (profiles/*pmc_traffic.json)
    when they were measured on this build and on this workload (traffic_tag: the passes' "config"
    field; None = the headline configuration)."""
    dom_name = max(layers, key=lambda k: layers[k]["ms"] * layers[k]["launches_per_frame"])
    dom = layers[dom_name]
    peak = PEAK_F16_MFMA_TFLOPS / SPLIT_PASSES
    roofline = dict(bound="mfma", achieved=round(dom["tflops"], 2), peak=round(peak, 1),
                    unit="TFLOP/s", frac=round(dom["tflops"] / peak, 4), traffic=None,
                    kernel=dom_name, launch_ms=round(dom["ms"], 4),
                    kernel_rule="the layer with the largest HIP-event ms x launches per frame; ISTA D and "
                                "ISTA P are twins (same MACs, 5 launches each, times within ~3 %), and "
                                "rocprof's per-dispatch means may rank the other one first",
                    flop_per_launch=2 * dom["macs"],
                    note="achieved = algorithmic fp32 FLOPs (2 x MACs) of one launch / its mean "
                         "duration; peak = 2500 TFLOP/s dense fp16 MFMA / 3 split passes")

    # HBM bytes per launch of the same kernel from the committed PMC passes (FETCH_SIZE and
    # WRITE_SIZE, separate rocprofv3 runs, gfx950 read correction): scripts/pmc_traffic.py
    import glob
    tfiles = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")))
    tag = "" if traffic_tag is None else traffic_tag + "_"
    tfiles = [f for f in tfiles if re.fullmatch(r"r\d\d_" + tag + "pmc_traffic\.json", os.path.basename(f))]
    if tfiles:
        try:
            import hashlib
            tj = json.load(open(tfiles[-1]))
            tl = tj["layers"].get(dom_name)
            sha = hashlib.sha256(open(lib_mod.LIB_PATH, "rb").read()).hexdigest()
            roofline["traffic_source"] = os.path.relpath(tfiles[-1], ROOT)
            if tl and tj.get("lib_sha256") == sha:
                roofline["traffic"] = tl["hbm_bytes_per_launch"]
                # the same launch against the HBM roof: the ISTA / Dg convs move as many bytes
                # per FLOP as the two roofs balance, so their time is bounded by the sum of the
                # two fractions when staging / epilogue and MFMAs do not overlap
                gbps = tl["hbm_bytes_per_launch"] / (dom["ms"] * 1e-3) / 1e9
                roofline["hbm_achieved_GBps"] = round(gbps, 1)
                roofline["hbm_frac"] = round(gbps / (HBM_TBPS * 1e3), 4)
                # the same PMC run's SQ / GRBM counters of that kernel (rNN_pmc_counters.json,
                # scripts/pmc_summary.py): the clock the chip held over the launch (GRBM_GUI_ACTIVE
                # / 8 XCDs / duration) and the matrix pipes' busy share of those cycles; the peak
                # above assumes 2.4 GHz, the convs run power-limited below it
                cfile = tfiles[-1].replace("pmc_traffic.json", "pmc_counters.json")
                if os.path.exists(cfile):
                    ck = tl["kernel"].replace("conv3x3_split3<", "conv<").replace(" ", "")
                    cv = json.load(open(cfile)).get(ck)
                    if cv and cv.get("GRBM_GUI_ACTIVE") and cv.get("dur_us"):
                        clk = cv["GRBM_GUI_ACTIVE"] / 8 / (cv["dur_us"] * 1e3)
                        roofline["pmc_counters_source"] = os.path.relpath(cfile, ROOT)
                        roofline["clock_ghz_held"] = round(clk, 3)
                        roofline["mfma_busy"] = round(cv["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (cv["GRBM_GUI_ACTIVE"] / 8), 4)
                        roofline["frac_at_held_clock"] = round(roofline["frac"] * 2.4 / clk, 4)
            else:       # measured on another build (or not this kernel): never quote stale bytes
                roofline["traffic_note"] = ("no PMC traffic of this build's " + dom_name + " kernel in "
                                            + roofline["traffic_source"])
        except (OSError, ValueError, KeyError):
            pass

    return roofline


def host_cores():
    """Threads for a cpu_baseline leg (every core the process may run on): all of
    os.sched_getaffinity, capped by the cgroup's CPU quota (cpu.max) when there is one -- the
    cores actually granted -- and by OMP_NUM_THREADS only when that is set explicitly.  Returns
    (threads, note naming the three numbers)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    n = aff if quota is None else min(aff, quota)
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    note = (f"{n} threads of {aff} affine cores (cgroup quota {quota if quota else 'none'}, "
            f"OMP_NUM_THREADS {omp if omp else 'unset'})")
    return n, note


def psnr(a, b):
    """utils/evaluate.py:18-28 (PIXEL_MAX = 1, 100 if mse < 1e-10)."""
    import numpy as np
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    return 100.0 if mse < 1e-10 else 20 * math.log10(1.0 / math.sqrt(mse))


def cpu_baseline(torch, model, vox, H, W, n_frames, timed=None, n_last=3, min_s=10.0, max_seqs=24):
    """Bounded CPU sample of the same workload: the reference's forward restated op for op on
    ATen's CPU kernels (oracle/cista_oracle_torch.py -- what the reference itself runs on a
    CPU), multi-threaded over this process's host cores, on B=1 sequences of n_frames recurrent
    frames at full size, repeated until >= min_s seconds (at most max_seqs sequences).

    Also returns the agreement (PSNR of utils/evaluate.py:18-28, max relative errors) of the
    TIMED path's own frames with the CPU restatement on the same inputs: `timed` = the frames
    the timed region produced for sequences 0 and B-1, (L, 2, 1, H, W) on the host (the
    whole-sequence graph replay at the bench batch, with its two-region tiling and XCD item
    order), against CPU sequence 0 over n_frames frames and CPU sequence B-1 over n_last frames.
    Without `timed` (eager-only runs) the comparison falls back to an eager B=1 run of
    sequence 0."""
    import numpy as np
    from oracle import fixtures as fx
    from oracle.cista_oracle_torch import CistaLSTCTorchCPU
    cores, core_note = host_cores()
    torch.set_num_threads(cores)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    ref = CistaLSTCTorchCPU(fx.collapse_tied(sd, model.depth), model.depth)
    L, B = vox.shape[0], vox.shape[1]
    n_frames = min(n_frames, L)
    ref.run_sequence(vox[:1, :1].cpu().numpy())                 # warm-up (oneDNN primitives)
    frames, dt, seqs, o_recs = 0, 0.0, 0, None
    while seqs < min(max_seqs, B) and (dt < min_s or seqs == 0):
        v = vox[:n_frames, seqs:seqs + 1].cpu().numpy()
        t0 = time.perf_counter()
        recs, _ = ref.run_sequence(v)
        dt += time.perf_counter() - t0
        if o_recs is None:
            o_recs = recs
        frames += n_frames
        seqs += 1
    pairs = []                      # (GPU frames, CPU frames), each (n, 1, 1, H, W)
    if timed is not None:
        pairs.append((np.asarray(timed[:n_frames, :1]), o_recs))
        n_last = min(n_last, L)
        last_ref, _ = ref.run_sequence(vox[:n_last, B - 1:B].cpu().numpy())
        pairs.append((np.asarray(timed[:n_last, 1:2]), last_ref))
        what = (f"the timed graph replay's frames of sequence 0 ({n_frames} frames) and sequence {B - 1} "
                f"({n_last} frames) at B={B}")
    else:
        with torch.no_grad():
            prev = torch.zeros(1, 1, H, W, device=vox.device)
            states = None
            g_recs = []
            for f in range(n_frames):
                prev, states = model(vox[f, :1], prev, states)
                g_recs.append(prev.cpu().numpy())
        pairs.append((np.stack(g_recs), o_recs))
        what = f"an eager B=1 run of sequence 0 ({n_frames} frames)"
    rel = max(float(np.abs(g - o).max() / np.abs(o).max()) for g, o in pairs)
    # SURVEY 7's frame metric: per pixel, each against its own magnitude
    erel = max(float((np.abs(g.astype(np.float64) - o) / np.maximum(np.abs(o), 1e-30)).max()) for g, o in pairs)
    ps = float(np.mean([psnr(g[f], o[f]) for g, o in pairs for f in range(len(o))]))
    return dict(value=frames / dt, unit="frames/s", cores=int(cores), kind="port",
                sample=f"{seqs} sequence(s) x {n_frames} recurrent frames at {H}x{W} (B=1), "
                       f"PyTorch-CPU op-for-op restatement (oracle/cista_oracle_torch.py), "
                       f"{core_note}, {dt:.1f} s"), ps, rel, erel, what


def frame_work(lib_mod, model, H, W):
    """Algorithmic work of one frame (B = 1) of this model config: MACs summed over the frame's
    layers (the library's cista_layer_macs, SURVEY 2.3 closed form; 22 793 011 200 at 180x240,
    C=64, depth 5, 5 bins) and HBM bytes 4*H*W*(num_bins + 2 + 3C) (voxel, prev
    image, states in and out, frame)."""
    L = lib_mod.lib()
    cfg = model._cfg()
    macs = 0.0
    for lid, name in enumerate(lib_mod.LAYERS):
        macs += L.cista_layer_macs(ctypes.byref(cfg), lid, 1, H, W) * (model.depth if name.startswith("ista") else 1)
    return macs, 4 * H * W * (model.num_bins + 2 + 3 * model.base_channels)


def time_steps(torch, fn, steps, warmup, vd=None, device=None):
    """Seconds for `steps` calls of fn after `warmup`, bracketed by barrier + synchronize."""
    for _ in range(warmup):
        out = fn()
    torch.cuda.synchronize()
    if vd is not None:
        vd.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    if vd is not None:
        vd.barrier()
    return time.perf_counter() - t0, out


def batch_sweep(torch, model, args, device, batches):
    """Small-batch / latency sweep (B in {1, 8, 32, 64, 128}): per batch size the
    per-frame latency (one recurrent frame of B sequences) and frames/s, eager per-frame module
    calls and the whole-sequence hipGraph replay; rank 0 only, a few sequences each."""
    from v2e2v_amd.sequence import CistaSequence
    H, W, L = args.height, args.width, args.len_seq
    out = {}
    for B in batches:
        vox = synth_voxels(torch, L, B, model.num_bins, H, W, args.num_events, seed=5000 + B, device=device)
        steps = 8 if B <= 8 else 3
        with torch.no_grad():
            te, _ = time_steps(torch, lambda: run_sequence(torch, model, vox, B, H, W, device), steps, 1)
            seq = CistaSequence(model, vox)
            tg, _ = time_steps(torch, seq.run, steps, 1)
            seq.close()
        out[str(B)] = {"frame_ms_eager": round(te / (steps * L) * 1e3, 4),
                       "frame_ms_graph": round(tg / (steps * L) * 1e3, 4),
                       "frames_per_s_eager": round(B * L * steps / te, 1),
                       "frames_per_s_graph": round(B * L * steps / tg, 1)}
        del vox
    return out


def pg_info(vd):
    """The ranks the process group actually holds and its backend (nccl = RCCL on ROCm); a
    single process without a launcher has no group: 1 rank, None."""
    import torch.distributed as dist
    return {"ranks_seen": dist.get_world_size() if vd.active() else 1,
            "process_group": dist.get_backend() if vd.active() else None}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, poll_s=0.2):
    """bench.py --gpus N (N > 1) started without a rank launcher: N fresh child interpreters
    running this script, one rank per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N, MASTER_* on
    127.0.0.1, and the launcher marker v2e2v_amd.dist reads), the role torchrun plays for the
    driver's scaling runs.  The parent never touches the GPU and never execs: it waits on its
    children, and as soon as one fails it stops the others (their exact PIDs) so no rank is
    left waiting in a collective.  Returns the exit code: 0 only if every rank exited 0.
    Replaces the reference's single-GPU picker (train_e2v.py:3-14, test_e2v.py:2-13)."""
    import signal
    import subprocess
    from v2e2v_amd.dist import LAUNCHER_ENV
    port = str(_free_port())

    def die_with_parent():
        # in the child, before it runs anything: SIGTERM when the launcher dies (Linux prctl
        # PR_SET_PDEATHSIG), so a launcher killed from outside leaves no rank holding a GPU
        try:
            import ctypes as _ct
            _ct.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)
        except OSError:
            pass

    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env[LAUNCHER_ENV] = "bench.py"
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      preexec_fn=die_with_parent))

    def forward(signum, _frame):            # a terminated launcher stops its ranks first
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        raise SystemExit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    rc = 0
    try:
        while [p.poll() for p in procs].count(None):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            time.sleep(poll_s)
        else:
            rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc != 0:
        print(f"bench.py: a rank failed (exit {rc}); {n}-rank run aborted", file=sys.stderr)
    return 0 if rc == 0 else (rc if rc > 0 else 128 - rc)


def rank_plan(args):
    """How this process takes part: ("launch", N) -- start N ranks (launch_ranks); ("rank", N) --
    one rank of an N-rank job set up by a launcher (torchrun or launch_ranks); ("single", 1).
    A launcher's WORLD_SIZE must agree with --gpus when both are given: a mismatch raises
    SystemExit(2), so a scaling run can never report the wrong number of GPUs."""
    from v2e2v_amd import dist as vd
    world = int(os.environ.get("WORLD_SIZE", "1"))
    launched = vd.under_launcher() or world > 1
    if launched:
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} "
                             f"ranks; refusing to report a {world}-rank run as {args.gpus} GPUs")
        args.gpus = world
        return "rank", world
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}")
    args.gpus = n
    return ("launch", n) if n > 1 else ("single", 1)


def dry_run_main(args, vd):
    """--dry-run: the rank plumbing alone, on CPU over gloo (no HIP call): barrier, K timed
    trivial steps, max over ranks, rank 0 prints the line the real bench would shape."""
    import torch
    import torch.distributed as dist
    if os.environ.get("V2E2V_DRY_FAIL_RANK") == os.environ.get("RANK", "0"):
        raise SystemExit(3)         # test hook: this rank dies before the process group forms
    rank, world, _ = vd.init("gloo")
    x = torch.ones(4096)
    vd.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = x * 1.0001
    vd.barrier()
    elapsed = vd.max_over_ranks(time.perf_counter() - t0)
    pids = [os.getpid()]
    if vd.active():
        pids = [None] * world
        dist.all_gather_object(pids, os.getpid())
    if rank == 0:
        print(json.dumps({"metric": "launcher dry run (no GPU work)", "value": round(world * args.steps / max(elapsed, 1e-9), 2),
                          "unit": "steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ranks_seen": dist.get_world_size() if vd.active() else 1,
                          "process_group": dist.get_backend() if vd.active() else None,
                          "rank_pids": pids}), flush=True)
    vd.finalize()


def main():
    args = parse()
    role, n = rank_plan(args)
    if role == "launch":
        sys.exit(launch_ranks(n, sys.argv[1:]))
    from v2e2v_amd import dist as vd
    if args.dry_run:
        return dry_run_main(args, vd)
    import torch
    from v2e2v_amd import CistaLSTCNet, _lib
    from v2e2v_amd.sequence import CistaSequence

    rank, world, local_rank = vd.env_rank()
    if world > 1 and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: {world} ranks but {torch.cuda.device_count()} visible GPU(s)")
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    vd.init("nccl", device)
    if args.mode == "train":
        return train_main(args, torch, vd, rank, world, device)
    if args.mode == "v2e2v":
        return v2e2v_main(args, torch, vd, rank, world, device)
    B, L, H, W = args.batch, args.len_seq, args.height, args.width
    nb, C, depth = args.num_bins, args.base_channels, args.depth

    model = CistaLSTCNet([H, W], base_channels=C, depth=depth, num_bins=nb)
    he_init_(torch, model, seed=7)
    model = model.to(device).eval()
    macs_frame, bytes_frame = frame_work(_lib, model, H, W)
    # sequences of this rank: a disjoint shard (seed offset by rank)
    vox = synth_voxels(torch, L, B, nb, H, W, args.num_events, seed=1000 + rank, device=device)
    torch.cuda.synchronize()

    # timed region: K steps of the L-frame recurrence over resident voxels, either as eager
    # per-frame module calls (the reference harness's loop) or as one hipGraph replay per step
    timings = {}
    with torch.no_grad():
        if args.graph in ("auto", "off"):
            timings["eager"] = time_steps(torch, lambda: run_sequence(torch, model, vox, B, H, W, device),
                                          args.steps, args.warmup, vd, device)
        if args.graph in ("auto", "on"):
            seq = CistaSequence(model, vox)
            timings["graph"] = time_steps(torch, lambda: seq.run()[0][-1], args.steps, args.warmup, vd, device)
    # the max over ranks of each path; the headline is the graph replay whenever it was timed
    # (a fixed choice: taking the faster of two short timings would bias the metric upwards)
    el = {k: vd.max_over_ranks(v[0], device) for k, v in timings.items()}
    path = "graph" if "graph" in el else "eager"
    elapsed = el[path]
    rec = timings[path][1]
    rec = rec[0] if isinstance(rec, tuple) else rec
    finite = bool(torch.isfinite(rec).all())
    # the timed replay's own frames of the first and last sequence (every frame of the last
    # replay; each step replays the same inputs), kept for the parity check against the CPU path
    timed_recs = seq.recs[:, [0, B - 1]].cpu().numpy() if path == "graph" else None
    frames = world * B * L * args.steps
    value = frames / elapsed

    layers = time_layers(torch, model, _lib, vox, B, H, W, device, args.layer_reps)
    roofline = dominant_roofline(layers, _lib)

    voxelizer = (time_voxelizer(torch, B * L, args.num_events, nb, H, W, device,
                                cpu_leg=world == 1 and not args.no_cpu_baseline) if rank == 0 else None)

    cpu = None
    psnr_vs_ref = rel_vs_ref = erel_vs_ref = parity_sample = None
    if world == 1 and not args.no_cpu_baseline:       # the CPU leg: rank 0 at N=1 only
        cpu, psnr_vs_ref, rel_vs_ref, erel_vs_ref, parity_sample = cpu_baseline(
            torch, model, vox, H, W, min(args.cpu_frames, L), timed=timed_recs)

    if rank == 0:
        frame_ms = sum(v["ms"] * v["launches_per_frame"] for v in layers.values())
        sweep = None
        if args.sweep and world == 1:         # single-GPU side measurement
            sweep = batch_sweep(torch, model, args, device, [int(x) for x in args.sweep.split(",") if x])
        cfg_name = f"{H}x{W} {nb}-bin depth={depth} C={C}"
        out = {
            "metric": "reconstructed frames/sec/GPU at 180x240 5-bin depth=5; PSNR vs ref"
                      if (H, W, nb, depth, C) == (180, 240, 5, 5, 64)
                      else f"reconstructed frames/sec/GPU at {cfg_name}; PSNR vs ref",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            **pg_info(vd),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (GPU-generated 15000-event voxels; He-scaled random-init weights)",
            "config": {"workload": f"CISTA-LSTC inference {cfg_name}, "
                                   f"len_sequence={L}, {B} sequences/GPU",
                       "timed_path": "whole-sequence hipGraph replay (v2e2v_amd/sequence.py)"
                                     if path == "graph" else "eager per-frame CistaLSTCNet.forward",
                       "batch_per_gpu": B, "len_sequence": L, "height": H, "width": W,
                       "num_events": args.num_events, "parallelism": f"replicas x{world}",
                       "precision": "split3-f16 MFMA (fp32 accumulate)"},
            "frames_per_s_per_gpu": round(value / world, 2),
            "tflops_effective": round(value * 2 * macs_frame / 1e12, 2),
            "eager_vs_graph_frames_per_s": {k: round(frames / v, 1) for k, v in el.items()},
            # whole-path fractions of BASELINE.md's roofline framing, per GPU: algorithmic FLOPs
            # and bytes per frame x frames/s over the peak
            "path_fractions": {
                "mfma_frac_vs_split3_peak": round(value / world * 2 * macs_frame
                                                  / (PEAK_F16_MFMA_TFLOPS / SPLIT_PASSES * 1e12), 4),
                "mfma_frac_vs_fp32_matrix_peak": round(value / world * 2 * macs_frame
                                                       / (PEAK_F32_MFMA_TFLOPS * 1e12), 4),
                "hbm_frac": round(value / world * bytes_frame / (HBM_TBPS * 1e12), 5),
                "hbm_gbps_algorithmic": round(value / world * bytes_frame / 1e9, 1)},
            "psnr_vs_ref": None if psnr_vs_ref is None else round(psnr_vs_ref, 2),
            "max_rel_err_vs_ref": rel_vs_ref,
            "max_elementwise_rel_err_vs_ref": erel_vs_ref,
            "parity_sample": parity_sample,
            "outputs_finite": finite,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "layers_ms": {k: round(v["ms"], 4) for k, v in layers.items()},
            "layers_tflops": {k: round(v["tflops"], 1) for k, v in layers.items()},
            "sum_of_kernels_ms_per_frame_batch": round(frame_ms, 3),
            "voxelizer": voxelizer,
            "batch_sweep": sweep,
        }
        print(json.dumps(out), flush=True)
    vd.finalize()


if __name__ == "__main__":
    main()
