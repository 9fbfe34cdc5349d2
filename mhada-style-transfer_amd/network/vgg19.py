"""Frozen VGG19 loss network — drop-in for ``MHAdaSTr/network/vgg19.py:15-70``.

The reference pulls ImageNet weights from torchvision at construction (a network fetch this
environment cannot make); here the layers are built with the same indices so a locally
saved ``slice{1..5}.{idx}.{weight,bias}`` state_dict loads strictly.  Forward = the training
path's loss features: on a ROCm device the HIP kernels (zero-pad Winograd / implicit-GEMM convs,
fused ReLU, max-pool, fused normalise; gradients flow to the input image), on the CPU aten.
"""
import torch.nn as nn

from . import _path  # noqa: F401
from mhada_hip import autograd_path

# torchvision vgg19 cfg "E" features[0:30]: (index, in, out) of each 3x3 conv; ReLU follows
# each conv, MaxPool2d(2) at 4, 9, 18, 27.
_CONVS = [(0, 3, 64), (2, 64, 64), (5, 64, 128), (7, 128, 128), (10, 128, 256), (12, 256, 256),
          (14, 256, 256), (16, 256, 256), (19, 256, 512), (21, 512, 512), (23, 512, 512), (25, 512, 512),
          (28, 512, 512)]
_POOLS = (4, 9, 18, 27)
_SLICES = ((0, 2), (2, 7), (7, 12), (12, 21), (21, 30))


class VGG19(nn.Module):
    def __init__(self):
        super().__init__()
        convs = {i: (ci, co) for i, ci, co in _CONVS}
        for s, (a, b) in enumerate(_SLICES, start=1):
            seq = nn.Sequential()
            for x in range(a, b):
                if x in convs:
                    seq.add_module(str(x), nn.Conv2d(convs[x][0], convs[x][1], 3, padding=1))
                elif x in _POOLS:
                    seq.add_module(str(x), nn.MaxPool2d(2, 2))
                else:
                    seq.add_module(str(x), nn.ReLU(inplace=True))
            setattr(self, f"slice{s}", seq)
        for p in self.parameters():
            p.requires_grad = False

    def forward(self, x):
        return autograd_path.vgg19_forward(self, x)

    def load_torchvision_features(self, src) -> None:
        """ImageNet weights from a LOCAL torchvision VGG19 checkpoint — the file that
        ``torchvision.models.vgg19(weights="VGG19_Weights.IMAGENET1K_V1")`` (vgg19.py:18) downloads
        (``vgg19-dcbb9e9d.pth``), a path to it or its state_dict: ``features.{i}.{weight,bias}``
        load into ``slice{s}.{i}`` (the reference keeps ``features[0:30]``, vgg19.py:20-36); the
        classifier and features past index 29 are ignored.  Loaded with ``weights_only=True``.
        Every conv of the five slices must be present (strict), shapes must match."""
        import torch
        sd = torch.load(src, map_location="cpu", weights_only=True) if not isinstance(src, dict) else src
        convs = {c[0] for c in _CONVS}
        own = {}
        for s, (a, b) in enumerate(_SLICES, start=1):
            for i in (x for x in range(a, b) if x in convs):
                for t in ("weight", "bias"):
                    key = f"features.{i}.{t}"
                    if key not in sd:
                        raise KeyError(f"load_torchvision_features: {key} missing")
                    own[f"slice{s}.{i}.{t}"] = sd[key]
        self.load_state_dict(own, strict=True)
