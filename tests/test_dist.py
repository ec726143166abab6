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


def _single_worker(port, q):
    # torchrun --nproc-per-node 1 sets the rank environment at world size 1: the process group
    # must still come up (the N=1 scaling point runs the same DDP all-reduce as N=8)
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      TORCHELASTIC_RUN_ID="test")
    r, w, _ = vd.init("gloo")
    up = vd.active()
    m = torch.nn.Linear(3, 2)
    net = torch.nn.parallel.DistributedDataParallel(m)
    net(torch.ones(4, 3)).sum().backward()
    g = m.weight.grad.clone()
    vd.barrier()
    vd.finalize()
    q.put((r, w, up, vd.active(), g.tolist()))


def test_world_size_one_under_launcher_initialises_process_group():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_single_worker, args=(_free_port(), q))
    p.start()
    r, w, up, after, g = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert (r, w, up, after) == (0, 1, True, False)
    assert g == [[4.0, 4.0, 4.0], [4.0, 4.0, 4.0]]      # DDP at world size 1: the all-reduce is exact


def test_no_process_group_without_launcher(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "TORCHELASTIC_RUN_ID", vd.LAUNCHER_ENV):
        monkeypatch.delenv(k, raising=False)
    assert not vd.under_launcher()
    assert vd.init("gloo") == (0, 1, 0)
    assert not vd.active()


def test_scheduler_rank_env_at_world_one_is_not_a_launcher(monkeypatch):
    """A scheduler / MPI wrapper that exports WORLD_SIZE=1 and MASTER_PORT is not torchrun:
    the process stays single-process (no TCPStore, no DDP wrap)."""
    for k in ("TORCHELASTIC_RUN_ID", vd.LAUNCHER_ENV):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("MASTER_PORT", "29999")
    assert not vd.under_launcher()
    assert vd.init("gloo") == (0, 1, 0)
    assert not vd.active()
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "x")
    assert vd.under_launcher()


def test_shard_partition_properties():
    for n in (0, 1, 7, 64, 65):
        for w in (1, 2, 3, 8):
            parts = [list(vd.shard(n, r, w)) for r in range(w)]
            flat = [i for p in parts for i in p]
            assert flat == list(range(n))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1


# ------------------------------------------------------------------ c4's data path
TINY = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_tiny")


def _tiny_dataset():
    import types
    from v2e2v_amd import data
    cfgs = types.SimpleNamespace(path_to_train_data=TINY, num_bins=5, image_dim=[24, 32], num_events=300,
                                 len_sequence=6, add_noise=False)
    return data.TrainFixNEventData(os.path.join(TINY, "train_e2v.txt"), cfgs)


def _seq_of(ds, events):
    """Sequence index of a raw item: its first event's time is the line number of its first line
    (tests/golden/make_train_tiny.py)."""
    first_line = int(round(float(events[0, 0])))
    return [s[0][0] for s in ds.sequence_line_id].index(first_line)


def _loader_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from v2e2v_amd import data
    vd.init("gloo")
    ds = _tiny_dataset()
    res = {}
    # per-rank batch 1: the rank's shard through the DataLoader (raw items; the GPU voxelisation
    # of GpuVoxelLoader.__iter__ is not run on CPU), rank and world from the process group
    ld = data.GpuVoxelLoader(ds, "cpu", batch_size=1)
    res["world"] = (ld.rank, ld.world_size, len(ld))
    res["plain"] = [_seq_of(ds, it[0][0]) for it in ld.loader]
    # world_size given without rank: the rank still comes from the process group (not 0 everywhere)
    res["ws_only_rank"] = data.GpuVoxelLoader(ds, "cpu", batch_size=1, world_size=world).rank
    ld = data.GpuVoxelLoader(ds, "cpu", batch_size=1, shuffle=True, seed=5)
    for ep in (0, 1):
        ld.set_epoch(ep)
        res[f"shuf{ep}"] = [_seq_of(ds, it[0][0]) for it in ld.loader]
    # per-rank batch 2: rank 0's first batch pairs a 6-frame and a 5-frame sequence -> refused
    ld = data.GpuVoxelLoader(ds, "cpu", batch_size=2)
    try:
        next(iter(ld))
        res["ragged"] = "accepted"
    except RuntimeError as e:
        res["ragged"] = "refused" if "equal size" in str(e) else repr(e)
    gathered = [None] * world
    torch.distributed.all_gather_object(gathered, res)
    q.put((rank, gathered))
    torch.distributed.destroy_process_group()


def test_gloo_loader_shards_are_disjoint_and_cover_the_split():
    world = 2
    ds = _tiny_dataset()
    assert len(ds) == 6 and sorted({len(s) for s in ds.sequence_line_id}) == [5, 6]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loader_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = res[0][1]
    assert [r["world"] for r in g] == [(0, 2, 3), (1, 2, 3)]
    for key in ("plain", "shuf0", "shuf1"):
        shards = [set(r[key]) for r in g]
        assert all(len(r[key]) == 3 for r in g)                 # same step count on every rank
        assert not (shards[0] & shards[1])                       # disjoint
        assert shards[0] | shards[1] == set(range(6))            # together the whole split
    assert g[0]["plain"] == [0, 2, 4] and g[1]["plain"] == [1, 3, 5]
    assert g[0]["shuf0"] != g[0]["shuf1"] or g[1]["shuf0"] != g[1]["shuf1"]   # reshuffled per epoch
    assert g[0]["ragged"] == "refused"                           # sequences 0 (6 frames) + 2 (5 frames)
    assert [r["ws_only_rank"] for r in g] == [0, 1]


def test_loader_needs_a_rank_for_world_size():
    """world_size > 1 with no rank and no process group would put every process on shard 0."""
    from v2e2v_amd import data
    ds = _tiny_dataset()
    with pytest.raises(ValueError):
        data.GpuVoxelLoader(ds, "cpu", batch_size=1, world_size=2)
    with pytest.raises(ValueError):
        data.GpuVoxelLoader(ds, "cpu", batch_size=1, world_size=2, rank=2)
    assert data.GpuVoxelLoader(ds, "cpu", batch_size=1, world_size=2, rank=1).rank == 1


def test_sequence_shard_sampler_properties():
    from v2e2v_amd.data import SequenceShardSampler
    for n in (0, 1, 6, 7, 64, 65):
        for w in (1, 2, 3, 8):
            for shuffle in (False, True):
                parts = []
                for r in range(w):
                    s = SequenceShardSampler(n, r, w, shuffle=shuffle, seed=1)
                    s.set_epoch(3)
                    parts.append(list(s))
                    assert len(parts[-1]) == len(s) == n // w
                flat = [i for p in parts for i in p]
                assert len(flat) == len(set(flat)) == (n // w) * w and set(flat) <= set(range(n))
    with pytest.raises(ValueError):
        SequenceShardSampler(4, 2, 2)
