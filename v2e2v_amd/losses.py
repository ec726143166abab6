"""Training losses on the GPU.

``SSIM`` / ``ssim`` mirror ``pytorch_msssim`` 0.2.1 (reference requirements.txt:10), the module
the reference's training loops build as ``SSIM(data_range=1, size_average=True, channel=1,
nonnegative_ssim=False)`` and use as ``loss_ssim = 1 - ssim_loss_fn(output, gt)``
(train_e2v.py:70,119; train.py:76,131).  The filtering, the SSIM map, its per-image mean and the
gradient with respect to the first argument run in libcista_hip.so (include/cista_loss.h);
``size_average`` and ``nonnegative_ssim`` are the library's host-side reductions, kept here in
torch so that autograd sees them.  The second argument (the ground truth) takes no gradient.

L1 stays ``torch.nn.L1Loss`` exactly as in the reference.  LPIPS needs VGG weights that are not
available offline; it is not provided.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

MAX_WIN = 31


class CistaSsimConfig(ctypes.Structure):
    _fields_ = [("win_size", ctypes.c_int), ("win", ctypes.c_float * MAX_WIN), ("data_range", ctypes.c_double),
                ("K1", ctypes.c_double), ("K2", ctypes.c_double)]


def _fspecial_gauss_1d(size: int, sigma: float) -> torch.Tensor:
    """pytorch_msssim 0.2.1 ``_fspecial_gauss_1d``: the same float32 CPU ops, so the same bits."""
    coords = torch.arange(size).to(dtype=torch.float)
    coords -= size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    g /= g.sum()
    return g


_ws: dict = {}


def _workspace(dev, nbytes):
    key = (dev.type, dev.index)
    b = _ws.get(key)
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        _ws[key] = b
    return b


def _config(win: torch.Tensor, data_range: float, K) -> CistaSsimConfig:
    cfg = CistaSsimConfig()
    n = win.numel()
    cfg.win_size = n
    vals = win.detach().to("cpu", torch.float32).flatten().tolist()
    for i in range(n):
        cfg.win[i] = vals[i]
    cfg.data_range = float(data_range)
    cfg.K1, cfg.K2 = float(K[0]), float(K[1])
    return cfg


class _SsimPerChannel(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, Y, win, data_range, K):
        if not X.is_cuda:
            raise _lib.CistaError("SSIM runs on a ROCm GPU only (no CPU fallback)")
        N, C, H, W = X.shape
        cfg = _config(win, data_range, K)
        Xc = X.detach().contiguous().float()
        Yc = Y.detach().contiguous().float()
        L = _lib.lib()
        ws = _workspace(X.device, L.cista_ssim_workspace_bytes(N, C, H, W, cfg.win_size))
        out = torch.empty(N, C, device=X.device, dtype=torch.float32)
        _lib.check(L.cista_ssim_forward(ctypes.byref(cfg), Xc.data_ptr(), Yc.data_ptr(), N, C, H, W, out.data_ptr(),
                                        None, ws.data_ptr(), ws.numel(), _lib.stream_handle(X.device)),
                   "cista_ssim_forward")
        ctx.save_for_backward(Xc, Yc)
        ctx.cfg = cfg
        return out

    @staticmethod
    def backward(ctx, g):
        Xc, Yc = ctx.saved_tensors
        N, C, H, W = Xc.shape
        cfg = ctx.cfg
        L = _lib.lib()
        ws = _workspace(Xc.device, L.cista_ssim_workspace_bytes(N, C, H, W, cfg.win_size))
        gX = torch.empty_like(Xc)
        gc = g.detach().contiguous().float()
        _lib.check(L.cista_ssim_backward(ctypes.byref(cfg), Xc.data_ptr(), Yc.data_ptr(), N, C, H, W, gc.data_ptr(),
                                         gX.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle(Xc.device)),
                   "cista_ssim_backward")
        return gX, None, None, None, None


def ssim(X, Y, data_range=255, size_average=True, win_size=11, win_sigma=1.5, win=None, K=(0.01, 0.03),
         nonnegative_ssim=False):
    """pytorch_msssim.ssim (0.2.1) for 4-d (N, C, H, W) inputs."""
    if not X.shape == Y.shape:
        raise ValueError("Input images should have the same dimensions.")
    if len(X.shape) != 4:
        raise ValueError(f"Input images should be 4-d tensors, but got {X.shape}")
    if not X.type() == Y.type():
        raise ValueError("Input images should have the same dtype.")
    if win is not None:
        win_size = win.shape[-1]
    if not (win_size % 2 == 1):
        raise ValueError("Window size should be odd.")
    if win is None:
        win = _fspecial_gauss_1d(win_size, win_sigma)
    if Y.requires_grad:
        raise NotImplementedError("the ground-truth argument of SSIM takes no gradient in this build")
    ssim_per_channel = _SsimPerChannel.apply(X, Y, win.reshape(-1), data_range, K)
    if nonnegative_ssim:
        ssim_per_channel = torch.relu(ssim_per_channel)
    if size_average:
        return ssim_per_channel.mean()
    return ssim_per_channel.mean(1)


class SSIM(torch.nn.Module):
    """pytorch_msssim.SSIM (0.2.1) surface: same constructor arguments and defaults."""

    def __init__(self, data_range=255, size_average=True, win_size=11, win_sigma=1.5, channel=3, spatial_dims=2,
                 K=(0.01, 0.03), nonnegative_ssim=False):
        super().__init__()
        if spatial_dims != 2:
            raise NotImplementedError("only 2-d SSIM (the reference's use) is built")
        self.win_size = win_size
        self.win = _fspecial_gauss_1d(win_size, win_sigma).repeat([channel, 1] + [1] * spatial_dims)
        self.size_average = size_average
        self.data_range = data_range
        self.K = K
        self.nonnegative_ssim = nonnegative_ssim

    def forward(self, X, Y):
        return ssim(X, Y, data_range=self.data_range, size_average=self.size_average, win=self.win[0, 0],
                    K=self.K, nonnegative_ssim=self.nonnegative_ssim)
