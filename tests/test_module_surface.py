"""Drop-in boundary checks that need no GPU: the C-ABI library loads and exports every symbol
include/cista_lstc.h declares; the nn.Module surface (ctor, 45-key state_dict, tied weights,
checkpoint layout, init RNG stream) matches the reference; and the product path refuses to run
on CPU instead of falling back to anything."""
import ctypes
import os

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN
from v2e2v_amd import CistaLSTCNet, _lib


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    names = _lib.header_functions()
    assert len(names) >= 11
    for n in names:
        assert hasattr(L, n), n
    assert L.cista_abi_version() == 3
    for s in range(6):
        assert L.cista_status_string(s)


def test_sizes_and_invalid_config():
    L = _lib.lib()
    cfg = _lib.CistaConfig(64, 5, 5)
    assert L.cista_packed_bytes(ctypes.byref(cfg)) > 1404481 * 4 // 2
    assert L.cista_workspace_bytes(ctypes.byref(cfg), 2, 64, 64) > 0
    bad = _lib.CistaConfig(0, 5, 5)
    assert L.cista_packed_bytes(ctypes.byref(bad)) == 0
    assert L.cista_workspace_bytes(ctypes.byref(cfg), 0, 64, 64) == 0
    # host-side validation happens before any device work: no GPU needed
    io = _lib.CistaFrameIO()
    st = L.cista_forward(ctypes.byref(cfg), None, 1, 64, 64, ctypes.byref(io), None, 0, None)
    assert st == 1
    # W0 is computed inside the composed input stage for 1..8 bins (bench.py asks the build)
    W0, IN = _lib.LAYERS.index("W0"), _lib.LAYERS.index("input")
    assert L.cista_layer_fused(ctypes.byref(cfg), W0) == 1
    assert L.cista_layer_fused(ctypes.byref(cfg), IN) == 0
    assert L.cista_layer_fused(ctypes.byref(_lib.CistaConfig(64, 5, 9)), W0) == 0
    # cista_backward reads only the cista_grad_io members the caller's struct has: a struct
    # shorter than the ABI-1 fields is refused before any device work
    fake = ctypes.c_void_p(256)
    prm = _lib.CistaParams(*([256] * 25))
    pg = _lib.CistaParamGrads(*([256] * 25))
    gio = _lib.CistaGradIO()
    saved = L.cista_saved_bytes(ctypes.byref(cfg), 1, 64, 64)
    assert L.cista_backward(ctypes.byref(cfg), fake, ctypes.byref(prm), 1, 64, 64, ctypes.byref(io), fake, saved,
                            ctypes.byref(gio), 16, ctypes.byref(pg), fake, 1 << 40, None) == 1
    odd = _lib.CistaConfig(48, 5, 5)   # base_channels % 32 != 0 -> unsupported, not wrong
    assert L.cista_forward(ctypes.byref(odd), ctypes.c_void_p(1), 1, 64, 64,
                           ctypes.byref(io), None, 0, None) == 2


def test_state_dict_layout_and_default_init_match_reference():
    ck = torch.load(os.path.join(GOLDEN, "f1_default.pth.tar"), weights_only=True)
    assert set(ck) == {"epoch", "state_dict"}
    torch.manual_seed(0)
    np.random.seed(0)
    m = CistaLSTCNet([64, 64], base_channels=64, depth=5, num_bins=5)
    sd = m.state_dict()
    assert list(sd) == list(ck["state_dict"])             # 45 keys, reference order
    assert len(sd) == 45
    for k, v in ck["state_dict"].items():
        assert sd[k].shape == v.shape
        assert torch.equal(sd[k], v), k                    # same RNG draws, same order
    assert sum(p.numel() for p in m.parameters()) == 1404481
    m.load_state_dict(ck["state_dict"], strict=True)


def test_tied_ista_last_copy_wins():
    m = CistaLSTCNet([32, 32], base_channels=32, depth=3, num_bins=5)
    sd = m.state_dict()
    sd = {k: v.clone() for k, v in sd.items()}
    sd["lista_blocks.0.Lambda"].fill_(1.0)
    sd["lista_blocks.2.Lambda"].fill_(7.0)
    m.load_state_dict(sd)
    assert m.lista_blocks[0] is m.lista_blocks[2]
    assert float(m.lista_blocks[0].Lambda.flatten()[0]) == 7.0


def test_cpu_tensors_raise_no_fallback():
    m = CistaLSTCNet([32, 32], base_channels=32, depth=1, num_bins=5)
    with torch.no_grad(), pytest.raises(RuntimeError, match="ROCm"):
        m(torch.zeros(1, 5, 32, 32), torch.zeros(1, 1, 32, 32), None)


def test_grad_mode_cpu_raises_no_fallback():
    """The training path (autograd + HIP backward) is GPU-only as well."""
    m = CistaLSTCNet([32, 32], base_channels=32, depth=1, num_bins=5)
    with pytest.raises(RuntimeError, match="ROCm"):
        m(torch.zeros(1, 5, 32, 32), torch.zeros(1, 1, 32, 32), None)


def test_voxelizer_surface_cpu():
    """The voxelizer has no CPU path: CPU input raises; argument errors mirror the reference's
    asserts (utils/event_process.py:22-25); invalid arguments are rejected by the C ABI."""
    from v2e2v_amd import event_process as ep
    from v2e2v_amd import _lib
    with pytest.raises(RuntimeError, match="ROCm"):
        ep.event_preprocess(torch.zeros(5, 8, 8))
    with pytest.raises(AssertionError):
        ep._as_events(np.zeros((3, 3)), torch.device("cpu"))
    L = _lib.lib()
    assert L.cista_voxelize(None, None, 1, 0, 0, 8, 8, 0, 0.0, None, None, 0, None) == 1
    assert L.cista_voxelize(None, None, 1, 0, 5, 8, 8, 7, 0.0, None, None, 0, None) == 1
    assert L.cista_voxel_preprocess(None, 1, 5, 8, 8, 3, 0.0, None, 0, None) == 1
    assert L.cista_voxelize(None, None, 0, 0, 5, 8, 8, 0, 0.0, None, None, 0, None) == 0   # B == 0: no-op


@pytest.mark.parametrize("block_px", [192, 96])
def test_two_region_tile_plan_invariants(block_px):
    """The forward convs' tiling (cista_tile_plan -> plan_tiles, host-only): over many output
    shapes the plan covers every row and column once (region a an exact multiple of its tile
    width, region b the remaining strip), never computes more tiles than the best one-region
    tiling, keeps each tile inside the workgroup's pixels and its halo inside the staging
    registers (4 items x 256 threads) and two LDS images per CU half; at 90 x 120 it cuts the
    192-pixel tiles from 60 to 57 and the 96-pixel ones from 115 to 113; and a
    launch of fewer than 1024 items keeps one region."""
    L = _lib.lib()
    rng = np.random.default_rng(block_px)
    shapes = [(90, 120), (60, 90), (45, 60), (360, 640), (1, 7), (7, 1), (16, 16), (33, 200)]
    shapes += [tuple(int(v) for v in rng.integers(1, 260, 2)) for _ in range(120)]
    out = (ctypes.c_int * 14)()
    for H, W in shapes:
        assert L.cista_tile_plan(256, H, W, block_px, out) == 0
        THa, TWa, tya, txa, msa, THb, TWb, tyb, txb, msb, wa, one, _, _ = list(out)
        for TH, TW, ty, tx, ms in ((THa, TWa, tya, txa, msa), (THb, TWb, tyb, txb, msb)):
            if tx == 0:
                continue
            assert ty * TH >= H and (ty - 1) * TH < H
            slots = TH * (16 * ms if ms else TW)
            assert TW >= 1 and slots <= block_px, (H, W, TH, TW, ms)
            halo = (TH + 2) * (TW + 2)
            assert ((halo + 7) & ~7) * 4 <= 4 * 256 and ((halo + 15) & ~15) * 128 * 2 <= 80 * 1024
        if txb == 0:
            assert wa == W and (txa - 1) * TWa < W <= txa * TWa
        else:
            assert 0 < wa < W and txa * TWa == wa
            assert (txb - 1) * TWb < W - wa <= txb * TWb
        assert tya * txa + tyb * txb <= one, (H, W)
    assert L.cista_tile_plan(256, 90, 120, block_px, out) == 0
    assert out[2] * out[3] + out[7] * out[8] == {192: 57, 96: 113}[block_px]
    assert out[11] == {192: 60, 96: 115}[block_px]
    assert L.cista_tile_plan(1, 90, 120, block_px, out) == 0          # 60 / 115 items: one round
    assert out[8] == 0 and out[10] == 120
    assert L.cista_tile_plan(256, 90, 120, 100, out) != 0
