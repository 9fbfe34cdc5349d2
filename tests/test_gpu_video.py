"""Video path: the per-style cache of the blocks' style-side tensors.

infer_video.py:58-92 computes fs = vit_s(style) once and calls adaFormer(fc, fs) per frame;
the build reuses each block's IN statistics, K|V' projection and V'^T image while the SAME fs
tensors come back unmodified.  Every test compares against a cache-off computation of the same
call (bit-identical: the cached tensors are the ones the cache-off path would compute)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import network
from mhada_hip.recipe import load_recipe, seeded_image

DEV = "cuda"


def models(act, dtype):
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(DEV).eval()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(DEV).eval()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(activation=act), "ada").to(DEV).eval()
    for m in (vc, vs, ada):
        m.compute_dtype = dtype
    return vc, vs, ada


def fresh(ada, fc, fs):
    ada.cache_style = False
    try:
        return ada(fc, fs)
    finally:
        ada.cache_style = True


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", ["softmax", "cosine"])
def test_cached_style_matches_uncached(act, dtype):
    vc, vs, ada = models(act, dtype)
    with torch.no_grad():
        fs = vs(seeded_image(1, 64, 96, 2).to(DEV))
        outs = []
        for seed in (3, 4, 5):  # three "frames" against one style
            fc = vc(seeded_image(1, 72, 128, seed).to(DEV))
            fcs, cs = ada(fc, fs)
            assert "_mhada_style" in ada.__dict__
            rfcs, rcs = fresh(ada, fc, fs)
            torch.testing.assert_close(cs, rcs, rtol=0, atol=0)
            torch.testing.assert_close(fcs, rfcs, rtol=0, atol=0)
            outs.append(cs)
        assert not torch.equal(outs[0], outs[1])


def test_cache_invalidated_by_inplace_edit_new_tensor_and_weights():
    vc, vs, ada = models("softmax", torch.float32)
    with torch.no_grad():
        fc = vc(seeded_image(1, 64, 64, 7).to(DEV))
        fs = vs(seeded_image(1, 64, 64, 8).to(DEV))
        ada(fc, fs)
        # in-place edit of a style feature bumps its version counter
        fs[1].mul_(1.5)
        _, cs = ada(fc, fs)
        _, rcs = fresh(ada, fc, fs)
        torch.testing.assert_close(cs, rcs, rtol=0, atol=0)
        # a new style whose buffers may reuse the freed allocation
        del fs
        fs2 = vs(seeded_image(1, 64, 64, 9).to(DEV))
        _, cs = ada(fc, fs2)
        _, rcs = fresh(ada, fc, fs2)
        torch.testing.assert_close(cs, rcs, rtol=0, atol=0)
        # a weight update of one block
        ada.adaAttnHead[3].g_list[2].weight.mul_(0.5)
        _, cs = ada(fc, fs2)
        _, rcs = fresh(ada, fc, fs2)
        torch.testing.assert_close(cs, rcs, rtol=0, atol=0)
