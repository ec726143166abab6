"""Whole-sequence hipGraph replay (v2e2v_amd/sequence.py, include/cista_lstc.h cista_sequence_*):
the graph replays exactly the kernels the eager module launches, so its frames and states must
be BIT-identical to the per-frame CistaLSTCNet loop of the reference harness
(test_e2v.py:105-117: prev_image = previous output, states carried)."""
import numpy as np
import pytest
import torch

from oracle import fixtures as fx
from v2e2v_amd import CistaLSTCNet
from v2e2v_amd.sequence import CistaSequence

pytestmark = pytest.mark.gpu
DEV = "cuda"


def model(H, W, seed=7):
    m = CistaLSTCNet([H, W])
    p = fx.stress_params(64, 5, 5, seed=seed)
    m.load_state_dict(fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in p.items()}, 5))
    return m.to(DEV).eval()


def eager(m, vox, prev, states):
    recs = []
    with torch.no_grad():
        for f in range(vox.shape[0]):
            prev, states = m(vox[f], prev, states)
            recs.append(prev)
    return torch.stack(recs), states


@pytest.mark.parametrize("B,H,W,L", [(1, 180, 240, 4), (3, 64, 96, 5)])
def test_graph_replay_bit_identical_to_eager(B, H, W, L):
    m = model(H, W)
    vox = torch.from_numpy(fx.synthetic_voxels(L, B, 5, H, W, n_events=fx.density_matched_events(H, W), seed=3)).to(DEV)
    seq = CistaSequence(m, vox)
    for _ in range(2):                                   # replays are repeatable
        recs, st = seq.run()
        torch.cuda.synchronize()
        ref, rst = eager(m, vox, torch.zeros(B, 1, H, W, device=DEV), None)
        assert torch.equal(recs, ref)
        for a, b in zip([st[0], st[1], st[2][0], st[2][1]], [rst[0], rst[1], rst[2][0], rst[2][1]]):
            assert torch.equal(a, b)
    # next sequence: new voxels in place, continuing from the last states and frame
    prev, states = recs[-1].clone(), [st[0].clone(), st[1].clone(), (st[2][0].clone(), st[2][1].clone())]
    seq2 = CistaSequence(m, vox, prev_image=prev, prev_states=states)
    vox.mul_(-0.5)
    r2 = seq2.run()[0].clone()           # run() returns its own (reused) buffers
    ref2, _ = eager(m, vox, prev, states)
    assert torch.equal(r2, ref2)
    # a parameter update is picked up (re-pack + re-capture)
    with torch.no_grad():
        m.final_conv.conv2d.bias.add_(0.25)
    r3, _ = seq2.run()
    ref3, _ = eager(m, vox, prev, states)
    assert torch.equal(r3, ref3) and not torch.equal(r3, r2)


def test_graph_replay_two_region_batch_bit_identical():
    """The bench's timed configuration in small: a whole-sequence graph replay at a batch where
    the forward convs tile in two regions (B=20 at 180x240: 20 x 57 items >= 1024, checked
    through cista_tile_plan) gives the eager B=20 loop's frames and states bit for bit, and
    each of its sequences equals that sequence run alone at B=1 (one region, small-batch tiles)."""
    import ctypes
    from v2e2v_amd import _lib
    B, H, W, L = 20, 180, 240, 3
    out = (ctypes.c_int * 14)()
    assert _lib.lib().cista_tile_plan(B, H // 2, W // 2, 192, out) == 0 and out[8] > 0      # region b present
    assert _lib.lib().cista_tile_plan(1, H // 2, W // 2, 192, out) == 0 and out[8] == 0     # B=1: one region
    m = model(H, W)
    vox = torch.from_numpy(fx.synthetic_voxels(L, B, 5, H, W, n_events=15000, seed=11)).to(DEV)
    seq = CistaSequence(m, vox)
    recs, st = seq.run()
    torch.cuda.synchronize()
    ref, rst = eager(m, vox, torch.zeros(B, 1, H, W, device=DEV), None)
    assert torch.equal(recs, ref)
    for a, b in zip([st[0], st[1], st[2][0], st[2][1]], [rst[0], rst[1], rst[2][0], rst[2][1]]):
        assert torch.equal(a, b)
    for s in (0, B - 1):
        one, ost = eager(m, vox[:, s:s + 1].contiguous(), torch.zeros(1, 1, H, W, device=DEV), None)
        assert torch.equal(recs[:, s:s + 1], one)
        assert torch.equal(st[1][s:s + 1], ost[1]) and torch.equal(st[2][1][s:s + 1], ost[2][1])


def test_bench_configuration_graph_replay_against_cpu_restatement():
    """The headline's timed configuration itself (bench.py: config c2, 180x240, 5 bins, depth 5,
    C=64, B=256 sequences, whole-sequence graph replay with the two-region tiling and XCD item
    order), 3 recurrent frames: the first and last sequences of the batch against the reference's
    forward restated on ATen's CPU kernels (oracle/cista_oracle_torch.py; pinned to the golden
    vectors), every pixel within 1e-4 of itself, states within 1e-4 of their max.
    Reference semantics: test_e2v.py:105-117 (prev_image = previous output, states carried)."""
    import bench
    from tests.conftest import elem_rel_err, rel_err
    from oracle.cista_oracle_torch import CistaLSTCTorchCPU
    B, H, W, L = 256, 180, 240, 3
    m = CistaLSTCNet([H, W])
    bench.he_init_(torch, m, seed=7)                      # the bench's own weights
    m = m.to(DEV).eval()
    vox = bench.synth_voxels(torch, L, B, 5, H, W, 15000, seed=1000, device=torch.device(DEV))
    seq = CistaSequence(m, vox)
    recs, st = seq.run()
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    ref = CistaLSTCTorchCPU(fx.collapse_tied(sd, 5), 5)
    for s in (0, B - 1):
        o_recs, o_st = ref.run_sequence(vox[:, s:s + 1].cpu().numpy())
        assert elem_rel_err(recs[:, s:s + 1].cpu().numpy(), o_recs) < 1e-4
        got = [st[0][s:s + 1], st[1][s:s + 1], st[2][0][s:s + 1], st[2][1][s:s + 1]]
        for g, r in zip(got, [o_st[0], o_st[1], o_st[2][0], o_st[2][1]]):
            assert rel_err(g.cpu().numpy(), r) < 1e-4
    seq.close()
