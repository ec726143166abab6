"""SSIM training loss on the GPU.

PARITY UNPINNED against pytorch_msssim itself (0.2.1, reference requirements.txt:10: absent here
and not vendored in the reference).  Forward: the HIP result against the numpy restatement
oracle/ssim_oracle.py in float64, bar 1e-5 relative (fp32 accumulation over 121-tap windows).
Backward: against torch autograd through a float64 torch restatement of the same algorithm,
bar 1e-4 of max|grad|.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import ssim_oracle as so
from tests.conftest import rel_err
from v2e2v_amd import losses

pytestmark = pytest.mark.gpu
FTOL, GTOL = 1e-5, 1e-4


def torch_ssim64(X, Y, data_range=1.0, K=(0.01, 0.03)):
    """float64 torch restatement (conv2d valid separable) used only as the autograd reference."""
    win = torch.from_numpy(so.gauss_1d(dtype=np.float64))
    C = X.shape[1]
    wv = win.view(1, 1, -1, 1).repeat(C, 1, 1, 1)
    wh = win.view(1, 1, 1, -1).repeat(C, 1, 1, 1)
    f = lambda t: F.conv2d(F.conv2d(t, wv, groups=C), wh, groups=C)
    C1, C2 = (K[0] * data_range) ** 2, (K[1] * data_range) ** 2
    mu1, mu2 = f(X), f(Y)
    s11 = f(X * X) - mu1 ** 2
    s22 = f(Y * Y) - mu2 ** 2
    s12 = f(X * Y) - mu1 * mu2
    cs = (2 * s12 + C2) / (s11 + s22 + C2)
    m = ((2 * mu1 * mu2 + C1) / (mu1 ** 2 + mu2 ** 2 + C1)) * cs
    return m.flatten(2).mean(-1)


def pair(shape, seed, noise=0.1):
    g = np.random.default_rng(seed)
    Y = g.uniform(0, 1, shape)
    X = np.clip(Y + g.normal(0, noise, shape), 0, 1)
    return X.astype(np.float32), Y.astype(np.float32)


@pytest.mark.parametrize("shape", [(8, 1, 180, 240), (2, 3, 40, 56), (1, 1, 11, 11), (3, 1, 23, 17)])
def test_forward_matches_restatement(shape):
    X, Y = pair(shape, sum(shape))
    got = losses.ssim(torch.from_numpy(X).cuda(), torch.from_numpy(Y).cuda(), data_range=1, size_average=False)
    ref, _ = so.ssim_per_channel(X.astype(np.float64), Y.astype(np.float64), 1.0)
    assert rel_err(got.cpu().numpy(), ref.mean(1)) < FTOL
    one = losses.ssim(torch.from_numpy(Y).cuda(), torch.from_numpy(Y).cuda(), data_range=1)
    assert abs(one.item() - 1.0) < 1e-5


@pytest.mark.parametrize("shape", [(4, 1, 64, 80), (2, 2, 30, 41)])
def test_backward_matches_autograd(shape):
    X, Y = pair(shape, 7 + shape[0])
    Xg = torch.from_numpy(X).cuda().requires_grad_(True)
    mod = losses.SSIM(data_range=1, size_average=True, channel=shape[1], nonnegative_ssim=False)
    loss = 1 - mod(Xg, torch.from_numpy(Y).cuda())
    loss.backward()
    X64 = torch.from_numpy(X.astype(np.float64)).requires_grad_(True)
    ref = 1 - torch_ssim64(X64, torch.from_numpy(Y.astype(np.float64))).mean()
    ref.backward()
    assert abs(loss.item() - ref.item()) <= FTOL * max(1.0, abs(ref.item()))
    assert rel_err(Xg.grad.cpu().numpy(), X64.grad.numpy()) < GTOL


def test_nonnegative_and_per_image_weights():
    X, Y = pair((3, 1, 32, 32), 3, noise=0.8)
    Xg = torch.from_numpy(X).cuda().requires_grad_(True)
    w = torch.tensor([1.0, -2.0, 0.5], device="cuda")
    (losses.ssim(Xg, torch.from_numpy(Y).cuda(), data_range=1, size_average=False, nonnegative_ssim=True)
     * w).sum().backward()
    X64 = torch.from_numpy(X.astype(np.float64)).requires_grad_(True)
    (torch.relu(torch_ssim64(X64, torch.from_numpy(Y.astype(np.float64))).mean(1)) * w.cpu().double()).sum().backward()
    assert rel_err(Xg.grad.cpu().numpy(), X64.grad.numpy()) < GTOL


def test_argument_errors_mirror_pytorch_msssim():
    a = torch.zeros(1, 1, 20, 20, device="cuda")
    with pytest.raises(ValueError):
        losses.ssim(a, torch.zeros(1, 1, 20, 21, device="cuda"))
    with pytest.raises(ValueError):
        losses.ssim(a, a, win_size=10)
    with pytest.raises(RuntimeError):
        losses.ssim(torch.zeros(1, 1, 8, 8, device="cuda"), torch.zeros(1, 1, 8, 8, device="cuda"))   # < win
