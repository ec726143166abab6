"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the SSIM training loss.

The reference's training loops use ``pytorch_msssim.SSIM(data_range=1, size_average=True,
channel=1, nonnegative_ssim=False)`` (reference train_e2v.py:27,70,119; train.py:23,76,131).
pytorch_msssim is a third-party dependency pinned at 0.2.1 (reference requirements.txt:10) that
is neither vendored in the reference nor installed here, so this restates its published
algorithm (``_fspecial_gauss_1d``, ``gaussian_filter``, ``_ssim``, ``ssim``): PARITY UNPINNED
against the library itself -- no reference fixture exercises it.  Only tests/ import this.
"""
from __future__ import annotations

import numpy as np


def gauss_1d(size: int = 11, sigma: float = 1.5, dtype=np.float32) -> np.ndarray:
    """_fspecial_gauss_1d: exp(-(c^2) / (2 sigma^2)) over c = arange(size) - size // 2, normalised."""
    c = np.arange(size).astype(dtype) - size // 2
    g = np.exp(-(c ** 2) / dtype(2 * sigma ** 2)).astype(dtype)
    return (g / g.sum()).astype(dtype)


def gaussian_filter(x: np.ndarray, win: np.ndarray) -> np.ndarray:
    """gaussian_filter: valid separable correlation, along H then along W; x (N, C, H, W)."""
    n = win.shape[0]
    H, W = x.shape[-2:]
    v = sum(win[k] * x[..., k:k + H - n + 1, :] for k in range(n))
    return sum(win[k] * v[..., :, k:k + W - n + 1] for k in range(n))


def ssim_per_channel(X: np.ndarray, Y: np.ndarray, data_range: float = 1.0, win: np.ndarray | None = None,
                     K=(0.01, 0.03)):
    """_ssim: (ssim_per_channel, cs) of shape (N, C), in X's dtype."""
    dt = X.dtype.type
    win = gauss_1d(dtype=dt) if win is None else win.astype(dt)
    C1 = dt((K[0] * data_range) ** 2)
    C2 = dt((K[1] * data_range) ** 2)
    mu1, mu2 = gaussian_filter(X, win), gaussian_filter(Y, win)
    mu1_sq, mu2_sq, mu1_mu2 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    s11 = gaussian_filter(X * X, win) - mu1_sq
    s22 = gaussian_filter(Y * Y, win) - mu2_sq
    s12 = gaussian_filter(X * Y, win) - mu1_mu2
    cs_map = (2 * s12 + C2) / (s11 + s22 + C2)
    ssim_map = ((2 * mu1_mu2 + C1) / (mu1_sq + mu2_sq + C1)) * cs_map
    N, C = X.shape[:2]
    return ssim_map.reshape(N, C, -1).mean(-1), cs_map.reshape(N, C, -1).mean(-1)


def ssim(X, Y, data_range=1.0, size_average=True, K=(0.01, 0.03), nonnegative_ssim=False):
    s, _ = ssim_per_channel(X, Y, data_range, None, K)
    if nonnegative_ssim:
        s = np.maximum(s, 0)
    return s.mean() if size_average else s.mean(1)
