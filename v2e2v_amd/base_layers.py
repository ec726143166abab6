"""Parameter containers with the reference's module names (e2v/base_layers.py).

They exist so that ``CistaLSTCNet.state_dict()`` has exactly the reference's 45 keys, in the
reference's order, with the reference's shapes and default initialisation (the same RNG draws
in the same order, so ``torch.manual_seed(s); np.random.seed(s)`` gives identical weights).
They hold parameters only: the computation is the fused HIP path in ``e2v_model.py``; none of
these classes has a forward.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
from torch.nn import Parameter


class _NoForward(nn.Module):
    def forward(self, *args, **kwargs):  # pragma: no cover - guard
        raise RuntimeError(f"{type(self).__name__} is a parameter container; call "
                           "CistaLSTCNet.forward (the fused MI355X path)")


def _check_norm(norm):
    if norm is not None:
        raise NotImplementedError("BN/IN norm branches are not on the CISTA-LSTC path "
                                  "(reference e2v/base_layers.py:147-150 with norm=None)")


class ConvLayer(_NoForward):
    """reference e2v/base_layers.py:135-161: conv2d(padding_mode='reflect') + activation."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 activation=None, norm=None):
        super().__init__()
        _check_norm(norm)
        self.conv2d = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding,
                                bias=True, padding_mode="reflect")
        self.activation = activation


class IstaBlock(_NoForward):
    """reference e2v/base_layers.py:21-35 (is_recurrent=False on this path: no gates conv)."""

    def __init__(self, base_channels=32, kernel_size=3, stride=1, padding=1):
        super().__init__()
        self.D = ConvLayer(2 * base_channels, base_channels, kernel_size, stride, padding)
        self.P = ConvLayer(base_channels, 2 * base_channels, kernel_size, stride, padding)
        # same draw as the reference (np.random.rand, :31) so seeds reproduce its init
        self.Lambda = Parameter(torch.tensor(0.001 * np.random.rand(1, 2 * base_channels, 1, 1),
                                             dtype=torch.float32))


class ConvLSTC(_NoForward):
    """reference e2v/base_layers.py:38-71; gates = (in, forget), out_gates, P0."""

    def __init__(self, x_size, z_size, output_size, kernel_size):
        super().__init__()
        pad = kernel_size // 2
        self.x_size, self.z_size, self.output_size = x_size, z_size, output_size
        self.gates = nn.Conv2d(x_size + z_size, 2 * output_size, kernel_size, padding=pad,
                               padding_mode="reflect")
        self.out_gates = nn.Conv2d(z_size + output_size, output_size, kernel_size, padding=pad,
                                   padding_mode="reflect")
        self.P0 = nn.Conv2d(x_size, output_size, kernel_size, padding=pad, padding_mode="reflect")


class ConvLSTM(_NoForward):
    """reference e2v/base_layers.py:75-130; Gates chunk order (in, remember, out, cell)."""

    def __init__(self, input_size, hidden_size, kernel_size):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        self.Gates = nn.Conv2d(input_size + hidden_size, 4 * hidden_size, kernel_size,
                               padding=kernel_size // 2, padding_mode="reflect")


class RecurrentConvLayer(_NoForward):
    """reference e2v/base_layers.py:214-225: ConvLayer + ConvLSTM."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=0,
                 activation=None, norm=None):
        super().__init__()
        self.conv = ConvLayer(in_channels, out_channels, kernel_size, stride, padding,
                              activation, norm)
        self.recurrent_block = ConvLSTM(out_channels, out_channels, 3)


class UpsampleConvLayer(_NoForward):
    """reference e2v/base_layers.py:166-210: bilinear x2 -> ReflectionPad2d(1) -> conv (pad 0)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 activation=None, norm=None):
        super().__init__()
        _check_norm(norm)
        self.pad = nn.ReflectionPad2d((kernel_size - 1) // 2)
        self.conv2d = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=True)
        self.activation = activation
