"""Pin the numpy oracle against golden vectors produced by the reference modules
(tests/golden/make_goldens.py).  CPU only."""
import numpy as np
import pytest
import torch

from mhada_hip.recipe import recipe_state_dict, seeded_image
from oracle import mhada_oracle as O
from conftest import load_golden

VIT_KEYS = None


def _vit_shapes(pos):
    shapes = {"patch_embedding.conv_proj.weight": (512, 3, 8, 8), "patch_embedding.conv_proj.bias": (512,)}
    if pos:
        shapes["pos_embedding.pos_embed"] = (1, 512, 32, 32)
    for i in range(3):
        p = f"encoder.{i}."
        shapes.update({p + "attention.in_proj_weight": (1536, 512), p + "attention.in_proj_bias": (1536,),
                       p + "attention.out_proj.weight": (512, 512), p + "attention.out_proj.bias": (512,),
                       p + "mlp.0.weight": (2048, 512), p + "mlp.0.bias": (2048,),
                       p + "mlp.2.weight": (512, 2048), p + "mlp.2.bias": (512,),
                       p + "ln1.weight": (512,), p + "ln1.bias": (512,),
                       p + "ln2.weight": (512,), p + "ln2.bias": (512,)})
    return shapes


def _block_shapes(pre=""):
    s = {}
    for i in range(8):
        for n in ("f", "g", "h"):
            s[f"{pre}{n}_list.{i}.weight"] = (64, 64, 1, 1)
            s[f"{pre}{n}_list.{i}.bias"] = (64,)
    s[f"{pre}out_conv.weight"] = (512, 512, 1, 1)
    s[f"{pre}out_conv.bias"] = (512,)
    return s


DEC = [("conv1.0", 512, 256), ("conv1.1", 256, 256), ("conv1.2", 256, 256), ("conv1.3", 256, 256),
       ("conv1.4", 256, 128), ("conv2.0", 128, 128), ("conv2.1", 128, 64), ("conv3.0", 64, 64),
       ("conv3.1", 64, 3)]


def _decoder_shapes(pre="decoder."):
    s = {}
    for name, ci, co in DEC:
        s[f"{pre}{name}.conv.conv.weight"] = (co, ci, 3, 3)
        s[f"{pre}{name}.conv.conv.bias"] = (co,)
    return s


def _ada_shapes():
    s = {}
    for k in range(6):
        s.update(_block_shapes(f"adaAttnHead.{k}."))
    s.update(_decoder_shapes())
    return s


def params(tag, shapes, dtype=np.float32):
    return O.to_numpy_params(recipe_state_dict(tag, shapes), dtype)


def rel_err(a, b):
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))


FULL_CASES = ["full_64_b1", "full_64_b2", "full_72x128_b3", "full_64x128_s64_b1", "cosine_64_b2", "full_256_b1"]


@pytest.mark.parametrize("case", FULL_CASES)
def test_oracle_full_forward_matches_reference(case):
    g = load_golden(case)
    cshape, sshape, seeds = g["content_shape"], g["style_shape"], g["seeds"]
    act = str(g["activation"])
    c = seeded_image(int(cshape[0]), int(cshape[1]), int(cshape[2]), int(seeds[0])).numpy()
    s = seeded_image(int(sshape[0]), int(sshape[1]), int(sshape[2]), int(seeds[1])).numpy()
    if "content" in g:
        np.testing.assert_array_equal(c, g["content"])  # input recipe is reproducible
    p_vc = params("vit_c", _vit_shapes(True))
    p_vs = params("vit_s", _vit_shapes(False))
    p_ada = params("ada", _ada_shapes())
    fc, fs, fcs, cs = O.stylize(c, s, p_vc, p_vs, p_ada, activation=act)
    for i in (0, 2):
        if f"fc{i}" in g:
            assert rel_err(fc[i], g[f"fc{i}"]) < 1e-4
            assert rel_err(fs[i], g[f"fs{i}"]) < 1e-4
    if "fcs" in g:
        assert rel_err(fcs, g["fcs"]) < 1e-4
    else:
        np.testing.assert_allclose(fcs.mean(axis=(2, 3)), g["fcs_mean"], rtol=1e-3, atol=1e-4)
        np.testing.assert_allclose(fcs[:, ::16, ::2, ::2], g["fcs_sub"], rtol=1e-3, atol=1e-3)
    # the contract metric: MSE on clamp(0,255)/255, far tighter here: fp32 vs fp32
    a = np.clip(cs, 0, 255) / 255.0
    b = np.clip(g["cs"], 0, 255) / 255.0
    assert float(((a - b) ** 2).mean()) < 1e-10
    assert float(np.abs(cs - g["cs"]).max()) < 5e-3


@pytest.mark.parametrize("case", ["block_b2_4x4_s3x5", "block_cos_b1_4x4"])
def test_oracle_block_matches_reference(case):
    g = load_golden(case)
    p = params("blk", _block_shapes())
    out = O.ada_attn_multihead(g["fc"], g["fs"], g["fcs"], p, "", 8, str(g["activation"]))
    assert rel_err(out, g["out"]) < 1e-5


def test_oracle_decoder_matches_reference():
    g = load_golden("decoder_b2_8x6")
    p = params("dec", _decoder_shapes())
    y = O.decoder_forward(g["x"], p)
    assert y.shape == g["y"].shape
    assert rel_err(y, g["y"]) < 1e-5


def test_oracle_interp_matches_torch():
    x = np.random.default_rng(0).standard_normal((2, 3, 5, 7)).astype(np.float32)
    for (oh, ow) in [(10, 14), (3, 4), (9, 16), (32, 32)]:
        ref = torch.nn.functional.interpolate(torch.from_numpy(x), size=(oh, ow), mode="bilinear",
                                              align_corners=False).numpy()
        np.testing.assert_allclose(O.interp_bilinear(x, oh, ow), ref, rtol=1e-5, atol=1e-6)
    ref = torch.nn.functional.interpolate(torch.from_numpy(x), scale_factor=2, mode="bilinear",
                                          align_corners=False).numpy()
    np.testing.assert_allclose(O.interp_bilinear(x, 10, 14, 0.5, 0.5), ref, rtol=1e-5, atol=1e-6)


def _vgg_shapes():
    import network
    return {k: tuple(v.shape) for k, v in network.VGG19().state_dict().items()}


def test_oracle_training_losses_match_reference():
    """Forward half of one train_image.py step (ViTs, AdaFormer x3, VGG19 x5, 4 losses)."""
    g = load_golden("train_64_b2")
    c = seeded_image(2, 64, 64, int(g["content_seed"])).numpy()
    s = seeded_image(2, 64, 64, int(g["style_seed"])).numpy()
    p = [params("vit_c", _vit_shapes(True)), params("vit_s", _vit_shapes(False)), params("ada", _ada_shapes()),
         params("vgg", _vgg_shapes())]
    losses = O.train_losses(c, s, *p)
    np.testing.assert_allclose(losses, g["losses"], rtol=2e-4)
    fc = O.vgg19_forward(c, p[3])
    np.testing.assert_allclose(fc["relu3_1"], g["vgg_fc_relu3_1"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(fc["relu5_1"], g["vgg_fc_relu5_1"], rtol=1e-4, atol=1e-5)
    fs = O.vgg19_forward(s, p[3])
    t4 = O.ada_attn_for_loss(fc["relu4_1"], fs["relu4_1"], O.feature_down_sample(fc, 4), O.feature_down_sample(fs, 4))
    np.testing.assert_allclose(t4, g["lf_target4"], rtol=1e-4, atol=1e-4)


def test_oracle_warp_functions_match_reference():
    """utilities.warp (both paddings), flow_warp_mask and the exps_sintel warping error."""
    g = load_golden("video_warp")
    for pad in ("zeros", "border"):
        np.testing.assert_allclose(O.warp(g["x"], g["flow"], pad), g[f"warp_{pad}"], rtol=0, atol=1e-3)
    np.testing.assert_array_equal(O.flow_warp_mask(g["flo01"], g["flo10"]), g["mask"])
    err = O.warping_error(g["cs1"], g["cs2"], g["flow"][:1], g["mask"][None])
    np.testing.assert_allclose(err, [g["warp_err"]], rtol=1e-5)


def test_temporal_losses_match_reference():
    """lossfn.output/feature_level_temporal_loss restated in mhada_hip.losses (autograd form)."""
    from mhada_hip import losses as L
    g = load_golden("video_warp")
    t = {k: torch.from_numpy(g[k]) for k in ("c1", "c2", "cs1", "cs2", "flow", "mask", "f1", "f2")}
    mse = torch.nn.MSELoss(reduction="none")
    m = t["mask"].unsqueeze(0)
    out = L.output_level_temporal_loss(t["c1"], t["c2"], t["cs1"] * 255, t["cs2"] * 255, t["flow"][:1], m, mse)
    np.testing.assert_allclose(float(out), float(g["out_temporal"]), rtol=1e-5)
    feat = L.feature_level_temporal_loss(t["f1"], t["f2"], t["flow"][:1], m, mse)
    np.testing.assert_allclose(float(feat), float(g["feat_temporal"]), rtol=1e-5)
