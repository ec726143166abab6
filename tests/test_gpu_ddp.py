"""Data-parallel training over RCCL's stand-in on one GPU (SURVEY section 8 row e, config c4;
reference train_e2v.py:92-130 trains on one GPU, north_star shards its batch over ranks).

Two ranks (spawned child processes, gloo backend, both on cuda:0) wrap CistaLSTCNet in
DistributedDataParallel and run the 3-frame BPTT of tests/golden/grads_32x48.npz (g2:
prev_img = output.clone(), states carried, L1 on the last frame), each on its own sample of
the fixture's B=2 batch.  DDP averages the per-rank gradients, which must reproduce the
single-process B=2 reference gradients (the L1 mean over 2 samples is the mean of the two
per-sample means), and one Adam step must leave both ranks with bit-identical parameters
and packed MFMA weights.  bench.py --mode train runs the same DDP path over RCCL ("nccl").
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


def _worker_c4(rank, world, port, out_dir):
    """Config c4's per-rank shape: 180x240, 5 frames (tests/golden/g4_spec.py), the fixture's B=8
    batch split over 2 ranks of B=4."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import hashlib

    import torch
    import torch.distributed as dist

    from oracle import fixtures as fx
    from tests.golden.g4_spec import G4, g4_inputs, g4_params
    from v2e2v_amd import CistaLSTCNet

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    c = G4
    per = c["B"] // world
    m = CistaLSTCNet([c["H"], c["W"]], base_channels=c["C"], depth=c["depth"], num_bins=5)
    sd = fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in g4_params().items()}, c["depth"])
    m.load_state_dict(sd, strict=True)
    m = m.to(dev).train()
    net = torch.nn.parallel.DistributedDataParallel(m, device_ids=[0], broadcast_buffers=False)
    vox_all, target_all = g4_inputs()
    vox = torch.from_numpy(np.ascontiguousarray(vox_all[:, rank * per:(rank + 1) * per])).to(dev)
    target = torch.from_numpy(np.ascontiguousarray(target_all[rank * per:(rank + 1) * per])).to(dev)
    prev = torch.zeros(per, 1, c["H"], c["W"], device=dev)
    state = None
    for s in range(c["L"]):
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


def test_ddp_c4_per_rank_shape_matches_fp64_truth(tmp_path, golden):
    """2 ranks x B=4 at 180x240 x 5 frames, DDP-wrapped, on one GPU: the all-reduced gradients
    equal the B=8 gradients of the fp64 reference within the single-process c3 bar
    (tests/test_gpu_train.py), and one Adam step leaves the replicas bit-identical."""
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_worker_c4, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [np.load(tmp_path / f"rank{i}.npz") for i in range(world)]
    d = golden("grads_180x240_b8.npz")
    bad = {}
    for key in [k for k in r[0].files if k.startswith("grad_")]:
        g0, g1 = r[0][key], r[1][key]
        assert np.array_equal(g0, g1), f"{key}: the all-reduced gradients differ between ranks"
        name = key[5:]
        e = rel_err(g0, d[f"f64_param_{name}"])
        bar = max(4 * float(d[f"noise32_param_{name}"]), 5e-4)
        if not e <= bar:
            bad[name] = (e, bar)
    assert not bad, bad
    mean_loss = (float(r[0]["loss"]) + float(r[1]["loss"])) / 2
    assert abs(mean_loss - float(d["f64_loss"])) <= 1e-4 * abs(float(d["f64_loss"]))
    assert np.array_equal(r[0]["params"], r[1]["params"])
    assert str(r[0]["packed_sha"]) == str(r[1]["packed_sha"])
