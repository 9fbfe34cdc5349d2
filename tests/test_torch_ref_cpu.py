"""Pin tests/torch_ref.py (the GPU tests' full-size reference) against the reference goldens."""
import numpy as np
import pytest
import torch

import network
import torch_ref
from conftest import load_golden
from mhada_hip.recipe import load_recipe, seeded_image


def sds():
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").state_dict()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").state_dict()
    return vc, vs


@pytest.mark.parametrize("case", ["full_64_b2", "full_64x128_s64_b1", "cosine_64_b2"])
def test_torch_ref_matches_goldens(case):
    g = load_golden(case)
    act = str(g["activation"])
    vc, vs = sds()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(activation=act), "ada").state_dict()
    cshape, sshape, seeds = g["content_shape"], g["style_shape"], g["seeds"]
    c = seeded_image(*map(int, cshape), int(seeds[0]))
    s = seeded_image(*map(int, sshape), int(seeds[1]))
    with torch.no_grad():
        fc, fs, fcs, cs = torch_ref.stylize(c, s, vc, vs, ada, act)
    np.testing.assert_allclose(cs.numpy(), g["cs"], rtol=1e-4, atol=2e-3)
    np.testing.assert_allclose(fcs.numpy(), g["fcs"], rtol=1e-4, atol=1e-3)
