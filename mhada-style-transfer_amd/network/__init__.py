"""Drop-in replacement for MHAdaSTr/network/ (reference ``network/__init__.py:1-3``) running
on MI355X HIP kernels.  Same class names, constructor signatures, forward signatures and
state_dict keys; reference checkpoints load with ``load_state_dict(strict=True)``.

    from network import VisionTransformer, AdaAttnTransformerMultiHead, AdaAttnForLoss, VGG19

Compute dtype: fp32 by default; bf16 under ``torch.autocast("cuda", dtype=torch.bfloat16)``
or with ``module.compute_dtype = torch.bfloat16``.
"""
from .adaDecoder import AdaAttnForLoss, AdaAttnMultiHead, AdaAttnTransformerMultiHead
from .conv import Decoder
from .vgg19 import VGG19
from .vit import VisionTransformer

__all__ = ["VisionTransformer", "AdaAttnTransformerMultiHead", "AdaAttnMultiHead", "AdaAttnForLoss",
           "Decoder", "VGG19"]
