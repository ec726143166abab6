"""Data-parallel training over RCCL's stand-in on one GPU (SURVEY section 8 row e, config c4;
reference train_e2v.py:92-130 trains on one GPU, north_star shards its batch over ranks).

Two ranks (spawned child processes, gloo backend, both on cuda:0) wrap CistaLSTCNet in
DistributedDataParallel and run the 3-frame BPTT of tests/golden/grads_32x48.npz (g2:
prev_img = output.clone(), states carried, L1 on the last frame), each on its own sample of
the fixture's B=2 batch.  DDP averages the per-rank gradients, which must reproduce the
single-process B=2 reference gradients (the L1 mean over 2 samples is the mean of the two
per-sample means), and one Adam step must leave both ranks with bit-identical parameters
and packed MFMA weights.  bench.py --mode train runs the same DDP path over RCCL ("nccl").

Config c4's own per-rank shape (B=8 at 180x240) runs as 2 gloo ranks x B=8 against a
single-process B=16 step, and one real RCCL ("nccl") rank at world size 1 -- what torchrun
--nproc-per-node 1 gives bench.py --mode train -- must reproduce the unwrapped model's gradients
bit for bit (test_nccl_world_size_one_ddp_gradients_bit_identical).
"""
import os
import socket
import sys

import numpy as np
import pytest

from tests.conftest import GOLDEN, ROOT, rel_err

pytestmark = pytest.mark.gpu
GTOL = 2e-4           # the single-process gradient bar of tests/test_gpu_train.py


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import hashlib

    import torch
    import torch.distributed as dist

    from oracle import fixtures as fx
    from v2e2v_amd import CistaLSTCNet

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    d = np.load(os.path.join(GOLDEN, "grads_32x48.npz"))
    C, depth = 64, 5
    m = CistaLSTCNet([32, 48], base_channels=C, depth=depth, num_bins=5)
    params = fx.stress_params(C, depth, 5, seed=21, lam=0.05)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, depth)
    m.load_state_dict(sd, strict=True)
    m = m.to(dev).train()
    net = torch.nn.parallel.DistributedDataParallel(m, device_ids=[0], broadcast_buffers=False)
    vox = torch.from_numpy(np.ascontiguousarray(d["voxels"][:, rank:rank + 1])).to(dev)
    target = torch.from_numpy(np.ascontiguousarray(d["g2_target"][rank:rank + 1])).to(dev)
    H, W = target.shape[-2:]
    prev = torch.zeros(1, 1, H, W, device=dev)
    state = None
    for s in range(3):
        out, state = net(vox[s], prev, state)
        prev = out.clone()
    loss = torch.nn.functional.l1_loss(out, target)
    loss.backward()
    torch.cuda.synchronize()
    grads = {k.replace("lista_blocks.0.", "lista."): p.grad.detach().cpu().numpy()
             for k, p in m.named_parameters()}
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    opt.step()
    packed = m.packed_params().cpu().numpy().tobytes()
    flat = np.concatenate([p.detach().cpu().numpy().ravel() for p in m.parameters()])
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), loss=np.float64(loss.item()),
             packed_sha=np.array(hashlib.sha256(packed).hexdigest()), params=flat,
             **{f"grad_{k}": v for k, v in grads.items()})
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_ddp_two_ranks_one_gpu_matches_single_process_gradients(tmp_path, golden):
    import torch.multiprocessing as mp
    world = 2
    # spawn: fresh interpreters started as child processes (the parent never execs)
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [np.load(tmp_path / f"rank{i}.npz") for i in range(world)]
    d = golden("grads_32x48.npz")
    bad = {}
    for key in [k for k in r[0].files if k.startswith("grad_")]:
        g0, g1 = r[0][key], r[1][key]
        assert np.array_equal(g0, g1), f"{key}: the all-reduced gradients differ between ranks"
        e = rel_err(g0, d[f"g2_f32_param_{key[5:]}"])
        if not e < GTOL:
            bad[key[5:]] = e
    assert not bad, bad
    # the per-rank losses average to the fixture's B=2 loss
    mean_loss = (float(r[0]["loss"]) + float(r[1]["loss"])) / 2
    assert abs(mean_loss - float(d["g2_f32_loss"])) <= 1e-4 * abs(float(d["g2_f32_loss"]))
    # one Adam step later both replicas hold the same parameters and the same packed weights
    assert np.array_equal(r[0]["params"], r[1]["params"])
    assert str(r[0]["packed_sha"]) == str(r[1]["packed_sha"])


def _c4_inputs(B):
    """Config c4's per-rank shape, 180x240 x 5 frames (tests/golden/g4_spec.py), for B sequences:
    sample b is seeded vox_seed + b (oracle/fixtures.synthetic_voxels), so samples 0..7 are the
    fixture's B=8 batch and 8..15 extend it."""
    from oracle import fixtures as fx
    from tests.golden.g4_spec import G4
    c = G4
    vox = fx.synthetic_voxels(c["L"], B, 5, c["H"], c["W"], n_events=15000, seed=c["vox_seed"])
    target = np.random.default_rng(c["target_seed"]).uniform(0, 1, (B, 1, c["H"], c["W"])).astype(np.float32)
    return vox, target


def _c4_model(dev):
    import torch

    from oracle import fixtures as fx
    from tests.golden.g4_spec import G4, g4_params
    from v2e2v_amd import CistaLSTCNet
    c = G4
    m = CistaLSTCNet([c["H"], c["W"]], base_channels=c["C"], depth=c["depth"], num_bins=5)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in g4_params().items()}, c["depth"])
    m.load_state_dict(sd, strict=True)
    return m.to(dev).train()


def _c4_bptt(net, vox, target, dev):
    import torch
    B = vox.shape[1]
    vox = torch.from_numpy(np.ascontiguousarray(vox)).to(dev)
    target = torch.from_numpy(np.ascontiguousarray(target)).to(dev)
    prev = torch.zeros(B, 1, target.shape[-2], target.shape[-1], device=dev)
    state = None
    for s in range(vox.shape[0]):
        out, state = net(vox[s], prev, state)
        prev = out.clone()
    loss = torch.nn.functional.l1_loss(out, target)
    loss.backward()
    torch.cuda.synchronize()
    return float(loss.item())


C4_PER_RANK = 8       # config c4: batch 64 over 8 GPUs = 8 sequences per rank


def _worker_c4(rank, world, port, out_dir):
    """Config c4 per rank: B=8 sequences at 180x240 (5 frames), the B=16 batch split over 2 ranks."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import hashlib

    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    per = C4_PER_RANK
    m = _c4_model(dev)
    net = torch.nn.parallel.DistributedDataParallel(m, device_ids=[0], broadcast_buffers=False)
    vox_all, target_all = _c4_inputs(world * per)
    loss = _c4_bptt(net, vox_all[:, rank * per:(rank + 1) * per], target_all[rank * per:(rank + 1) * per], dev)
    grads = {k.replace("lista_blocks.0.", "lista."): p.grad.detach().cpu().numpy()
             for k, p in m.named_parameters()}
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    opt.step()
    packed = m.packed_params().cpu().numpy().tobytes()
    flat = np.concatenate([p.detach().cpu().numpy().ravel() for p in m.parameters()])
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), loss=np.float64(loss),
             packed_sha=np.array(hashlib.sha256(packed).hexdigest()), params=flat,
             **{f"grad_{k}": v for k, v in grads.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_c4_b8_per_rank_matches_single_process_b16(tmp_path, golden):
    """Config c4's per-rank shape: 2 ranks x B=8 at 180x240 x 5 frames, DDP-wrapped, on one GPU.
    The all-reduced gradients equal a single-process B=16 BPTT step of the same GPU path (DDP's
    average of two B=8 mean-loss gradients is the B=16 mean-loss gradient), rank 0's loss is the
    fp64 reference loss of the fixture's B=8 batch (its samples 0..7), and one Adam step leaves the
    replicas bit-identical."""
    import torch
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_worker_c4, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [np.load(tmp_path / f"rank{i}.npz") for i in range(world)]
    d = golden("grads_180x240_b8.npz")
    assert abs(float(r[0]["loss"]) - float(d["f64_loss"])) <= 1e-4 * abs(float(d["f64_loss"]))
    dev = torch.device("cuda", 0)
    m = _c4_model(dev)
    vox, target = _c4_inputs(world * C4_PER_RANK)
    loss16 = _c4_bptt(m, vox, target, dev)
    ref = {k.replace("lista_blocks.0.", "lista."): p.grad.detach().cpu().numpy() for k, p in m.named_parameters()}
    del m
    torch.cuda.empty_cache()
    bad = {}
    for key in [k for k in r[0].files if k.startswith("grad_")]:
        g0, g1 = r[0][key], r[1][key]
        assert np.array_equal(g0, g1), f"{key}: the all-reduced gradients differ between ranks"
        e = rel_err(g0, ref[key[5:]])
        if not e < GTOL:
            bad[key[5:]] = e
    assert not bad, bad
    mean_loss = (float(r[0]["loss"]) + float(r[1]["loss"])) / 2
    assert abs(mean_loss - loss16) <= 1e-5 * abs(loss16)
    assert np.array_equal(r[0]["params"], r[1]["params"])
    assert str(r[0]["packed_sha"]) == str(r[1]["packed_sha"])


def _worker_nccl1(_idx, port, out_dir):
    """One RCCL ("nccl") rank at world size 1, as torchrun --nproc-per-node 1 runs bench.py
    --mode train: the DDP-wrapped 3-frame BPTT step must give the unwrapped model's gradients
    bit for bit (the all-reduce over one rank divides by 1)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      TORCHELASTIC_RUN_ID="test")
    sys.path.insert(0, ROOT)
    import torch

    from oracle import fixtures as fx
    from v2e2v_amd import CistaLSTCNet
    from v2e2v_amd import dist as vd

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    vd.init("nccl", dev)
    assert vd.active() and torch.distributed.get_backend() == "nccl"
    d = np.load(os.path.join(GOLDEN, "grads_32x48.npz"))
    C, depth = 64, 5
    params = fx.stress_params(C, depth, 5, seed=21, lam=0.05)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, depth)
    vox = torch.from_numpy(np.ascontiguousarray(d["voxels"])).to(dev)
    target = torch.from_numpy(np.ascontiguousarray(d["g2_target"])).to(dev)
    out_grads = {}
    for tag in ("plain", "ddp"):
        m = CistaLSTCNet([32, 48], base_channels=C, depth=depth, num_bins=5)
        m.load_state_dict(sd, strict=True)
        m = m.to(dev).train()
        net = m if tag == "plain" else torch.nn.parallel.DistributedDataParallel(
            m, device_ids=[0], broadcast_buffers=False)
        H, W = target.shape[-2:]
        prev = torch.zeros(target.shape[0], 1, H, W, device=dev)
        state = None
        for s in range(3):
            out, state = net(vox[s], prev, state)
            prev = out.clone()
        torch.nn.functional.l1_loss(out, target).backward()
        torch.cuda.synchronize()
        for k, p in m.named_parameters():
            out_grads[f"{tag}_{k}"] = p.grad.detach().cpu().numpy()
    vd.barrier()
    vd.finalize()
    np.savez(os.path.join(out_dir, "nccl1.npz"), **out_grads)


def test_nccl_world_size_one_ddp_gradients_bit_identical(tmp_path):
    import torch.multiprocessing as mp
    mp.start_processes(_worker_nccl1, args=(_free_port(), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    r = np.load(tmp_path / "nccl1.npz")
    names = [k[6:] for k in r.files if k.startswith("plain_")]
    assert len(names) == 25
    for n in names:
        assert np.array_equal(r[f"plain_{n}"], r[f"ddp_{n}"]), n
