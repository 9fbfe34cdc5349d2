"""Decoder — drop-in for ``MHAdaSTr/network/conv.py:23-100``.

Same module nesting as the reference (``conv1.0.conv.conv.weight`` ...).  On a ROCm device
``Decoder.forward`` runs the HIP convolutions (fp32: Winograd F(2x2,3x3); bf16: implicit-GEMM
MFMA and the 64->64 tile kernel with the bilinear x2 fused) and the dedicated Cin->3 output
kernel; CPU tensors run the aten form in ``mhada_hip.autograd_path``.
"""
import torch
import torch.nn as nn

from . import _path  # noqa: F401
from mhada_hip import autograd_path, engine


class Conv(nn.Module):
    """``conv.py:23-33``: ReflectionPad2d(k//2) + Conv2d (stride 1 on the hot path)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride)


class ConvReLU(nn.Module):
    """``conv.py:36-45``"""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int):
        super().__init__()
        self.conv = Conv(in_channels, out_channels, kernel_size, stride)


class ConvReluInterpolate(nn.Module):
    """``conv.py:61-72``: conv, ReLU, bilinear x scale_factor (align_corners=False)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int, scale_factor: float):
        super().__init__()
        self.conv = Conv(in_channels, out_channels, kernel_size, stride)
        self.scale_factor = scale_factor


class Decoder(nn.Module):
    """``conv.py:75-100``: 512@h -> 3@8h.  forward(fcs NCHW) -> cs NCHW fp32 (unclamped)."""

    def __init__(self):
        super().__init__()
        self.compute_dtype = None
        self.conv1 = nn.Sequential(
            ConvReluInterpolate(512, 256, 3, 1, 2),
            ConvReLU(256, 256, 3, 1),
            ConvReLU(256, 256, 3, 1),
            ConvReLU(256, 256, 3, 1),
            ConvReluInterpolate(256, 128, 3, 1, 2),
        )
        self.conv2 = nn.Sequential(
            ConvReLU(128, 128, 3, 1),
            ConvReluInterpolate(128, 64, 3, 1, 2),
        )
        self.conv3 = nn.Sequential(
            ConvReLU(64, 64, 3, 1),
            ConvReLU(64, 3, 3, 1),
        )

    def forward(self, fcs: torch.Tensor) -> torch.Tensor:
        if not fcs.is_cuda or autograd_path.needs_grad(self, fcs):  # autograd / CPU tensors
            return autograd_path.decoder_forward(self, fcs)
        dt = engine.resolve_compute_dtype(self)
        return engine.decoder_forward_tokens(self, engine.to_tokens(fcs), dt)
