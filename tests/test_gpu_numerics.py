"""Range and robustness of the split-fp16 MFMA path beyond the
std-normalised voxels of the other parity tests:

* unnormalised voxels (event_preprocess mode='none', reference utils/event_process.py:132-154,
  hot pixels kept) and weights scaled x1e-3: the frames and states stay within 1e-4 of the
  reference restatement (oracle/cista_oracle_torch.py, pinned to the golden vectors) and the
  range flag stays clear;
* weights scaled x3 and x100 drive the ISTA iterate to 3e6 / 1e23 in the fp32 reference, beyond
  what an fp16 hi part holds (|x| < 65504): the path must say so (range flag ->
  CistaError), never return silently wrong frames;
* NaN inputs propagate like torch.relu (not zeroed by the softshrink / ReLU epilogues);
* parameters written through `.data` are picked up after invalidate_packed().
"""
import numpy as np
import pytest
import torch

from oracle import fixtures as fx
from oracle.cista_oracle_torch import CistaLSTCTorchCPU
from tests.conftest import rel_err
from v2e2v_amd import CistaLSTCNet
from v2e2v_amd._lib import CistaError

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4
H = W = 64


def raw_voxels(n_frames=3, B=2, seed=3):
    """mode='none' voxels (no hot-pixel filter) with a hot pixel firing 400 events per window."""
    rng = np.random.default_rng(seed)
    vox = np.zeros((n_frames, B, 5, H, W), np.float32)
    for b in range(B):
        for f in range(n_frames):
            ev = fx.synthetic_events(fx.density_matched_events(H, W), H, W, rng)
            hot = np.stack([np.sort(rng.uniform(0, 0.05, 400)), np.full(400, 10.0 + b),
                            np.full(400, 20.0), np.ones(400)], 1)
            ev = np.concatenate([ev, hot])
            ev = ev[np.argsort(ev[:, 0], kind="stable")]
            vox[f, b] = fx.normalize_voxel(fx.voxelize(ev, 5, W, H), filter_hot_pixel=False, mode="none")
    return vox


def scaled_params(scale):
    p = fx.stress_params(64, 5, 5, seed=7)
    return {k: (v * np.float32(scale) if v.ndim == 4 else v) for k, v in p.items()}


def make_model(params):
    m = CistaLSTCNet([H, W], base_channels=64, depth=5, num_bins=5)
    m.load_state_dict(fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, 5),
                      strict=True)
    return m.to(DEV).eval()


def run_gpu(m, vox):
    B = vox.shape[1]
    prev = torch.zeros(B, 1, H, W, device=DEV)
    states = None
    recs = []
    with torch.no_grad():
        for f in range(vox.shape[0]):
            prev, states = m(torch.from_numpy(vox[f]).to(DEV), prev, states)
            recs.append(prev.cpu().numpy())
    torch.cuda.synchronize()
    return np.stack(recs), states


@pytest.mark.parametrize("scale", [1.0, 1e-3])
def test_unnormalised_voxels_and_small_weights_match_reference(scale):
    vox = raw_voxels()
    assert np.abs(vox).max() > 100                       # the hot pixel: far outside std-normalised range
    params = scaled_params(scale)
    m = make_model(params)
    recs, st = run_gpu(m, vox)
    m.check_numerics()                                   # flag clear
    ref_recs, ref_st = CistaLSTCTorchCPU(params, 5).run_sequence(vox)
    assert rel_err(recs, ref_recs) < TOL
    for got, ref in zip([st[0], st[1], st[2][0], st[2][1]], [ref_st[0], ref_st[1], ref_st[2][0], ref_st[2][1]]):
        assert rel_err(got.cpu().numpy(), ref) < TOL


@pytest.mark.parametrize("scale", [3.0, 100.0])
def test_out_of_range_activations_are_reported(scale):
    vox = raw_voxels()
    m = make_model(scaled_params(scale))
    # the forward's own asynchronous guard reports it a frame or two late, without a host sync
    # (run_gpu reads every frame back, so the flag's copy has landed by the next call)
    with pytest.raises(CistaError, match="65504"):
        run_gpu(m, np.concatenate([vox] * 3))
    # the synchronous check, with the asynchronous guard off
    m.range_check = False
    run_gpu(m, vox)
    with pytest.raises(CistaError, match="65504"):
        m.check_numerics()
    m.check_numerics()                                   # reported once, then cleared


def test_nan_input_propagates_like_torch():
    vox = fx.synthetic_voxels(1, 1, 5, H, W, n_events=fx.density_matched_events(H, W), seed=11)
    vox[0, 0, 2, 30, 30] = np.nan
    params = fx.stress_params(64, 5, 5, seed=7)
    m = make_model(params)
    recs, st = run_gpu(m, vox)
    ref_recs, _ = CistaLSTCTorchCPU(params, 5).run_sequence(vox)
    assert np.isnan(ref_recs).any()
    assert np.isnan(recs).any()                          # not silently zeroed by ReLU / softshrink
    assert np.isnan(st[1].cpu().numpy()).any()           # the ISTA iterate carries it


def test_packed_weights_follow_data_writes():
    vox = fx.synthetic_voxels(1, 1, 5, H, W, n_events=fx.density_matched_events(H, W), seed=12)
    params = fx.stress_params(64, 5, 5, seed=7)
    m = make_model(params)
    r0, _ = run_gpu(m, vox)
    lam = m.lista_blocks[0].Lambda
    lam.data.mul_(4.0)                                   # not version-counted by PyTorch
    m.invalidate_packed()
    r1, _ = run_gpu(m, vox)
    p2 = dict(params)
    p2["lista.Lambda"] = params["lista.Lambda"] * 4
    ref, _ = CistaLSTCTorchCPU(p2, 5).run_sequence(vox)
    assert rel_err(r1, ref) < TOL and not np.array_equal(r0, r1)
    # load_state_dict repacks by itself
    m.load_state_dict(fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}, 5))
    r2, _ = run_gpu(m, vox)
    assert np.array_equal(r2, r0)
