"""Multi-process (gloo, world_size 2, CPU) checks of the sequence sharding and the timing
reductions bench.py uses across ranks."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from v2e2v_amd import dist as vd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r, w, _ = vd.init("gloo")
    mine = list(vd.shard(37, r, w))
    got = torch.zeros(37)
    got[mine] = 1
    torch.distributed.all_reduce(got)
    mx = vd.max_over_ranks(float(r + 1))
    sm = vd.sum_over_ranks(float(len(mine)))
    vd.barrier()
    q.put((r, got.tolist(), mx, sm))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharding_and_reductions(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, got, mx, sm in res:
        assert got == [1.0] * 37          # every sequence on exactly one rank
        assert mx == float(world)
        assert sm == 37.0


def test_shard_partition_properties():
    for n in (0, 1, 7, 64, 65):
        for w in (1, 2, 3, 8):
            parts = [list(vd.shard(n, r, w)) for r in range(w)]
            flat = [i for p in parts for i in p]
            assert flat == list(range(n))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1
