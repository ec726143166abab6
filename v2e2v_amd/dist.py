"""Multi-GPU plumbing: one process per GPU (torchrun), sequences sharded across ranks.

Inference has no exchange step -- sequences are independent (no BN/IN), so each
rank reconstructs its own shard and nothing crosses xGMI on the data path.  The only
collectives are the benchmark's barrier and max-over-ranks timing (RCCL, or gloo on CPU for the
tests).  BPTT training wraps the module in DistributedDataParallel (one bucketed RCCL gradient
all-reduce per step, bench.py --mode train).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank():
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


LAUNCHER_ENV = "V2E2V_RANK_LAUNCHER"      # set by bench.py's own rank launcher (bench.py --gpus N)


def under_launcher() -> bool:
    """True when a rank launcher started this process -- torchrun / torch.distributed.run (its
    elastic agent exports TORCHELASTIC_RUN_ID to every worker) or bench.py's own --gpus N
    launcher (LAUNCHER_ENV) -- also at world size 1, where the process group still runs (one
    RCCL rank).  WORLD_SIZE / MASTER_PORT alone do not count: scheduler and MPI wrappers export
    those too, and a world-size-1 job under one of them stays single-process."""
    return "WORLD_SIZE" in os.environ and ("TORCHELASTIC_RUN_ID" in os.environ or LAUNCHER_ENV in os.environ)


def init(backend: str | None = None, device: torch.device | None = None):
    """Initialise the default process group when WORLD_SIZE > 1, or whenever the process was
    started by torchrun (WORLD_SIZE set, even to 1: the N=1 point of the scaling run then goes
    through the same RCCL process group and DDP all-reduce as N=8).  MASTER_ADDR=127.0.0.1."""
    rank, world, local = env_rank()
    if (world > 1 or under_launcher()) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def shard(n_items: int, rank: int, world: int) -> range:
    """Contiguous, balanced partition of n_items sequences; every item on exactly one rank."""
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def max_over_ranks(x: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def active() -> bool:
    """A process group is up (torchrun, any world size)."""
    return dist.is_available() and dist.is_initialized()


def finalize():
    if active():
        dist.destroy_process_group()
