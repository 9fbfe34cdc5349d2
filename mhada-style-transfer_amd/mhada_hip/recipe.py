"""Deterministic synthetic weights for the MHAdaSTr modules.

No trained checkpoint ships with the reference (``MHAdaSTr/models/models_save_path`` is a
placeholder), so every parity fixture, test and benchmark uses weights regenerated from this
recipe.  The recipe is keyed on the *state_dict key* so that the reference modules (loaded by
path in the golden generator) and this package's drop-in modules receive bit-identical
tensors through ``load_state_dict(strict=True)``.

Rules (applied per key, keys visited in sorted order, one CPU ``torch.Generator`` per key
seeded with ``crc32(tag + "." + key) ^ 0x5EED``):

* ``pos_embed``                         -> N(0, 0.02)   (``vit.py:79``, PosEmbedding init)
* LayerNorm ``ln{1,2}.weight / .bias``   -> 1 / 0        (``vit.py:54-55`` defaults)
* ``decoder.*`` conv weights             -> U(-sqrt(6/fan_in), +sqrt(6/fan_in))  (kaiming-ReLU;
  with PyTorch's default init the decoder output collapses to ~0.02 and pixel MSE becomes
  vacuous)
* every other weight                     -> U(-1/sqrt(fan_in), +1/sqrt(fan_in))
* every bias                             -> U(-1/sqrt(fan_in), +1/sqrt(fan_in)) of its weight

``tag`` distinguishes modules whose keys coincide (``vit_c`` / ``vit_s``).
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Tuple

import torch

_SEED_XOR = 0x5EED


def _generator(tag: str, key: str) -> torch.Generator:
    g = torch.Generator(device="cpu")
    g.manual_seed((zlib.crc32(f"{tag}.{key}".encode()) ^ _SEED_XOR) & 0xFFFFFFFF)
    return g


def _weight_key_for_bias(key: str) -> str:
    if key.endswith("in_proj_bias"):
        return key[: -len("in_proj_bias")] + "in_proj_weight"
    assert key.endswith("bias"), key
    return key[: -len("bias")] + "weight"


def _fan_in(shape: Tuple[int, ...]) -> int:
    return int(math.prod(shape[1:])) if len(shape) > 1 else int(shape[0])


def _is_layernorm(key: str) -> bool:
    parts = key.split(".")
    return len(parts) >= 2 and parts[-2] in ("ln1", "ln2")


def recipe_tensor(tag: str, key: str, shapes: Dict[str, Tuple[int, ...]]) -> torch.Tensor:
    shape = tuple(shapes[key])
    g = _generator(tag, key)
    t = torch.empty(shape, dtype=torch.float32)
    if key.endswith("pos_embed"):
        return t.normal_(0.0, 0.02, generator=g)
    if _is_layernorm(key):
        return t.fill_(1.0) if key.endswith("weight") else t.zero_()
    if key.endswith("bias"):
        wshape = tuple(shapes[_weight_key_for_bias(key)])
        bound = 1.0 / math.sqrt(_fan_in(wshape))
        return t.uniform_(-bound, bound, generator=g)
    fan_in = _fan_in(shape)
    if key.startswith("decoder.") or ".decoder." in key:
        bound = math.sqrt(6.0 / fan_in)
    else:
        bound = 1.0 / math.sqrt(fan_in)
    return t.uniform_(-bound, bound, generator=g)


def recipe_state_dict(tag: str, shapes: Dict[str, Tuple[int, ...]]) -> Dict[str, torch.Tensor]:
    """Return {key: fp32 CPU tensor} for every key in ``shapes`` (visited in sorted order)."""
    return {k: recipe_tensor(tag, k, shapes) for k in sorted(shapes)}


def load_recipe(module: torch.nn.Module, tag: str) -> torch.nn.Module:
    """Fill ``module`` (reference or drop-in) with the recipe weights, strict key match."""
    shapes = {k: tuple(v.shape) for k, v in module.state_dict().items()}
    sd = recipe_state_dict(tag, shapes)
    module.load_state_dict(sd, strict=True)
    return module


def seeded_image(batch: int, height: int, width: int, seed: int) -> torch.Tensor:
    """Synthetic image batch in the reference's [0, 255] float range (``toTensor255``,
    ``utilities.py:11-16``): ``torch.rand(B,3,H,W, generator=seed) * 255``."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    return torch.rand(batch, 3, height, width, generator=g) * 255.0
