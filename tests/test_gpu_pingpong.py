"""The two-tile ISTA convs (v2e2v_amd/csrc/cista_pingpong.hpp; reference e2v/e2v_model.py:72-78,
e2v/base_layers.py:11-12,21-35) against the one-tile kernel they replace at large batches:
frames and states bit for bit (same per-pixel arithmetic, same MFMA order), also when some tiles
overflow the fp16 hi part and go through the deferred range pass (conv3x3_fixup)."""
import numpy as np
import pytest
import torch

from oracle import fixtures as fx
from v2e2v_amd import CistaLSTCNet, _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(H, W, seed=7):
    m = CistaLSTCNet([H, W])
    p = fx.stress_params(64, 5, 5, seed=seed)
    m.load_state_dict(fx.expand_tied({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in p.items()}, 5))
    return m.to(DEV).eval()


def _run(m, vox, two_tile):
    lib = _lib.lib()
    prev = lib.cista_set_two_tile(3 if two_tile else 0)
    try:
        B, H, W = vox.shape[1], vox.shape[3], vox.shape[4]
        img = torch.zeros(B, 1, H, W, device=DEV)
        st = None
        recs = []
        with torch.no_grad():
            for f in range(vox.shape[0]):
                img, st = m(vox[f], img, st)
                recs.append(img)
        torch.cuda.synchronize()
        return torch.stack(recs), [st[0], st[1], st[2][0], st[2][1]]
    finally:
        lib.cista_set_two_tile(prev)


def _voxels(L, B, H, W, seed):
    # 2 distinct sequences tiled over the batch (numpy voxelisation of B sequences is slow)
    v = fx.synthetic_voxels(L, 2, 5, H, W, n_events=15000, seed=seed)
    return torch.from_numpy(np.ascontiguousarray(np.tile(v, (1, (B + 1) // 2, 1, 1, 1))[:, :B])).to(DEV)


def test_two_tile_bit_identical_to_one_tile():
    B, H, W = 80, 180, 240                   # 80 x 57 tiles: above the two-tile threshold
    m = _model(H, W)
    vox = _voxels(2, B, H, W, seed=31)
    vox[:, 1::2] *= -0.7                      # every sample distinct
    vox[:, 2::4] *= 1.3
    r1, s1 = _run(m, vox, True)
    r0, s0 = _run(m, vox, False)
    assert torch.equal(r1, r0)
    for a, b in zip(s1, s0):
        assert torch.equal(a, b)


def test_two_tile_overflow_tiles_take_the_range_pass():
    """Voxels x 1e4 in some samples: their ISTA inputs leave the fp16 range, the two-tile launch
    lists those tiles and conv3x3_fixup recomputes them (range pass) -- the same bits as the
    one-tile kernel's in-launch range pass; the other samples are untouched by it."""
    B, H, W = 80, 180, 240
    m = _model(H, W)
    vox = _voxels(2, B, H, W, seed=37)
    vox[:, 3] *= 1e4
    vox[:, 40] *= 3e4
    r1, s1 = _run(m, vox, True)
    r0, s0 = _run(m, vox, False)
    assert torch.isfinite(r1).all()
    assert torch.equal(r1, r0)
    for a, b in zip(s1, s0):
        assert torch.equal(a, b)
