"""MHAda blocks — drop-in for ``MHAdaSTr/network/adaDecoder.py:38-268``.

``AdaAttnMultiHead`` keeps the reference's per-head ``f_list/g_list/h_list`` 1x1 convs and
``out_conv`` (identical state_dict keys; the InstanceNorms and the activation modules carry
no state).  On a ROCm device the forward runs ``mhada_hip.engine.block_forward``: InstanceNorm
statistics kernel, per-batch weight fold, two grouped projection GEMMs, the fused flash-style
MHAda attention (M, S and S*IN(fcs)+M in its epilogue) and the out_conv GEMM.  CPU tensors (the
reference's no-GPU branch, ``infer_image.py:48``) run the aten form in ``autograd_path``.
"""
from typing import List

import torch
import torch.nn as nn

from . import _path  # noqa: F401
from mhada_hip import autograd_path, engine
from .conv import Decoder

ACTIVATIONS = ("softmax", "cosine")


def _check_activation(activation: str) -> str:
    if activation not in ACTIVATIONS:
        raise ValueError(f"Unknown activation function: {activation}")  # adaDecoder.py:50,160
    return activation


class AdaAttnForLoss(nn.Module):
    """Parameter-free AdaAttN used as the local-feature-loss target (``adaDecoder.py:38-81``).
    Training-path component: on a ROCm device the wide-head HIP kernel ``mhada_loss_attn``
    (qk_dim = 448..1472, d_v 256/512, A never stored); under autograd or on the CPU the
    reference expression with aten ops, query-chunked."""

    def __init__(self, v_dim, qk_dim, activation="softmax"):
        super().__init__()
        self.v_dim, self.qk_dim = v_dim, qk_dim
        self.activation_name = _check_activation(activation)

    def forward(self, c_x, s_x, c_1x, s_1x):
        return autograd_path.ada_attn_for_loss(c_x, s_x, c_1x, s_1x, self.activation_name)


class AdaAttnMultiHead(nn.Module):
    """``adaDecoder.py:134-206``: forward(fc, fs, fcs) -> (B, qkv_dim, h, w)."""

    def __init__(self, qkv_dim, num_heads, activation="softmax"):
        super().__init__()
        if qkv_dim % num_heads != 0:
            raise ValueError("qkv_dim 必須能被 num_heads 整除")  # adaDecoder.py:137-138 (same message)
        self.num_heads = num_heads
        self.head_dim = qkv_dim // num_heads
        self.compute_dtype = None
        self.f_list = nn.ModuleList([nn.Conv2d(self.head_dim, self.head_dim, kernel_size=1) for _ in range(num_heads)])
        self.g_list = nn.ModuleList([nn.Conv2d(self.head_dim, self.head_dim, kernel_size=1) for _ in range(num_heads)])
        self.h_list = nn.ModuleList([nn.Conv2d(self.head_dim, self.head_dim, kernel_size=1) for _ in range(num_heads)])
        self.out_conv = nn.Conv2d(qkv_dim, qkv_dim, kernel_size=1)
        self.activation_name = _check_activation(activation)

    def forward(self, fc: torch.Tensor, fs: torch.Tensor, fcs: torch.Tensor) -> torch.Tensor:
        if not fc.is_cuda or autograd_path.needs_grad(self, fc, fs, fcs):  # autograd / CPU tensors
            return autograd_path.block_forward(self, fc, fs, fcs)
        dt = engine.resolve_compute_dtype(self)
        fcf = engine._Feat.from_nchw(fc)
        fsf = engine._Feat.from_nchw(fs)
        fcsf = fcf if fcs is fc else engine._Feat.from_nchw(fcs)
        out = engine.block_forward(self, fcf, fsf, fcsf, dt)
        return engine.tokens_to_nchw(out.t, out.h, out.w)


class AdaAttnTransformerMultiHead(nn.Module):
    """``adaDecoder.py:235-268``: 2*num_layers MHAda blocks + Decoder.
    forward(fc_list, fs_list) or forward((fc_list, fs_list)) -> (fcs, cs)."""

    def __init__(self, num_layers: int = 3, qkv_dim: int = 512, num_heads: int = 8, activation: str = "softmax"):
        super().__init__()
        self.num_layers = num_layers
        self.compute_dtype = None
        self.adaAttnHead = nn.ModuleList(
            [AdaAttnMultiHead(qkv_dim=qkv_dim, num_heads=num_heads, activation=activation)
             for _ in range(num_layers * 2)])
        self.decoder = Decoder()

    def forward(self, *args):
        if len(args) == 1:
            fc, fs = args[0]
        else:
            fc, fs = args
        fc: List[torch.Tensor] = list(fc)
        fs: List[torch.Tensor] = list(fs)
        if not fc[0].is_cuda or autograd_path.needs_grad(self, *fc, *fs):  # autograd / CPU tensors
            return autograd_path.adaformer_forward(self, fc, fs)
        return engine.adaformer_forward(self, fc, fs)
