"""ViT content/style encoders — drop-in for ``MHAdaSTr/network/vit.py:45-169``.

Parameters live in the same torch containers the reference uses (``nn.Conv2d``,
``nn.MultiheadAttention``, ``nn.Linear``, ``nn.LayerNorm``) so the state_dict keys match
exactly.  On a ROCm device the forward never calls their aten forwards — it runs
``mhada_hip.engine.vit_forward`` (HIP kernels) for inference and the HIP training kernels under
autograd; CPU tensors (the reference's no-GPU branch, ``infer_image.py:48``) run the aten CPU
form in ``mhada_hip.autograd_path``.
"""
from typing import List

import torch
import torch.nn as nn

from . import _path  # noqa: F401
from mhada_hip import autograd_path, engine


class PosEmbedding(nn.Module):
    """``vit.py:67-102``: learned (1, C, 32, 32) table, bilinear-resized to the token grid."""

    def __init__(self, patch_size: int = 8, embed_dim: int = 512, base_embed_size: int = 32):
        super().__init__()
        self.patch_size = patch_size
        self.embed_dim = embed_dim
        self.base_embed_size = base_embed_size
        self.pos_embed = nn.Parameter(torch.empty(1, embed_dim, base_embed_size, base_embed_size).normal_(std=0.02))


class PatchEmbedding(nn.Module):
    """``vit.py:105-117``: conv k=s=patch, 3 -> hidden."""

    def __init__(self, in_channels: int, patch_size: int, hidden_dim: int):
        super().__init__()
        self.conv_proj = nn.Conv2d(in_channels, hidden_dim, kernel_size=patch_size, stride=patch_size)


class EncoderBlock(nn.Module):
    """``vit.py:45-64``: pre-LN (eps 1e-6) MHA over the batch axis + MLP 512-2048-512."""

    def __init__(self, num_heads: int, hidden_dim: int, mlp_dim: int):
        super().__init__()
        self.attention = nn.MultiheadAttention(embed_dim=hidden_dim, num_heads=num_heads)
        self.mlp = nn.Sequential(nn.Linear(hidden_dim, mlp_dim), nn.ReLU(), nn.Linear(mlp_dim, hidden_dim))
        self.ln1 = nn.LayerNorm(hidden_dim, eps=1e-6)
        self.ln2 = nn.LayerNorm(hidden_dim, eps=1e-6)


class VisionTransformer(nn.Module):
    """``vit.py:120-169``.  ``forward(x: (B,3,H,W)) -> [ (B,C,H/8,W/8) ] * num_layers``; the
    returned maps are NCHW views of token-major storage."""

    def __init__(self, patch_size: int = 8, num_layers: int = 3, num_heads: int = 8, hidden_dim: int = 512,
                 mlp_dim: int = 2048, pos_embedding: bool = True):
        super().__init__()
        self.patch_size = patch_size
        self.num_layers = num_layers
        self.hidden_dim = hidden_dim
        self.compute_dtype = None
        self.patch_embedding = PatchEmbedding(in_channels=3, patch_size=patch_size, hidden_dim=hidden_dim)
        self.pos_embedding = PosEmbedding(patch_size=patch_size, embed_dim=hidden_dim) if pos_embedding else None
        self.encoder = nn.ModuleList(
            [EncoderBlock(num_heads=num_heads, hidden_dim=hidden_dim, mlp_dim=mlp_dim) for _ in range(num_layers)])

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        # training / feature inversion (autograd over the HIP training kernels), or a CPU
        # tensor: infer_image.py:48 runs the modules on "cpu" when no GPU is present, and the
        # aten CPU form of the same expression serves that call
        if not x.is_cuda or autograd_path.needs_grad(self, x):
            return autograd_path.vit_forward(self, x)
        return engine.vit_forward(self, x)
