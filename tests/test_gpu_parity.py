"""End-to-end parity of the HIP forward path (network/ drop-in on MI355X).

* against the golden vectors produced by the reference modules (tests/golden/), all cases;
* against the numpy oracle on fresh seeded inputs (oracle/mhada_oracle.py);
* at BASELINE.json's full sizes against the plain-PyTorch fp32 restatement on the device.

Contract: pixel MSE on clamp(cs,0,255)/255 < 1e-4 for the fp32 and the bf16
paths; the fp32 path additionally has MSE < 1e-4 on the raw 0-255 scale.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import network
from conftest import load_golden
from mhada_hip.recipe import load_recipe, seeded_image

DEV = "cuda"
FULL_CASES = ["full_64_b1", "full_64_b2", "full_72x128_b3", "full_64x128_s64_b1", "cosine_64_b2", "full_256_b1"]


def models(act="softmax", dtype=torch.float32):
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(DEV).eval()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(DEV).eval()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(activation=act), "ada").to(DEV).eval()
    for m in (vc, vs, ada):
        m.compute_dtype = dtype
    return vc, vs, ada


def stylize(ms, c, s):
    vc, vs, ada = ms
    with torch.no_grad():
        fc = vc(c)
        fs = vs(s)
        fcs, cs = ada(fc, fs)
    return fc, fs, fcs, cs


def mse01(a, b):
    a = np.clip(np.asarray(a, dtype=np.float64), 0, 255) / 255.0
    b = np.clip(np.asarray(b, dtype=np.float64), 0, 255) / 255.0
    return float(((a - b) ** 2).mean())


def mse_raw(a, b):
    return float(((np.asarray(a, dtype=np.float64) - np.asarray(b, dtype=np.float64)) ** 2).mean())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", FULL_CASES)
def test_forward_matches_reference_goldens(case, dtype):
    g = load_golden(case)
    cshape, sshape, seeds = g["content_shape"], g["style_shape"], g["seeds"]
    c = seeded_image(*map(int, cshape), int(seeds[0])).to(DEV)
    s = seeded_image(*map(int, sshape), int(seeds[1])).to(DEV)
    fc, fs, fcs, cs = stylize(models(str(g["activation"]), dtype), c, s)
    cs = cs.cpu().numpy()
    assert cs.shape == g["cs"].shape
    assert mse01(cs, g["cs"]) < 1e-4
    if dtype == torch.float32:
        assert mse_raw(cs, g["cs"]) < 1e-4
        if "fcs" in g:
            np.testing.assert_allclose(fcs.cpu().numpy(), g["fcs"], rtol=1e-3, atol=2e-3)
        for i in (0, 2):
            if f"fc{i}" in g:
                np.testing.assert_allclose(fc[i].cpu().numpy(), g[f"fc{i}"], rtol=1e-3, atol=1e-3)
                np.testing.assert_allclose(fs[i].cpu().numpy(), g[f"fs{i}"], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("split", ["all", "none"])
@pytest.mark.parametrize("case", FULL_CASES)
def test_fp32_goldens_with_split3_forced(case, split, monkeypatch):
    """The fp32 path's two arithmetic forms against the reference goldens.  "all": every SPLIT3
    product forced on — the ViT's QKV / MLP1 / MLP2 GEMMs whatever the tile-fill rule
    (engine._split3_fills picks them only from ~30k tokens, more than any golden case has) and the
    SPLIT3 MHAda attention; "none": the fp32-MFMA kernels throughout.  Same bounds as the default
    fp32 run: pixel and raw MSE < 1e-4, fc / fs / fcs allclose."""
    from mhada_hip import engine, ops
    monkeypatch.setattr(engine, "_split3_fills", lambda M, N, dev: split == "all")
    monkeypatch.setattr(ops, "F32_SPLIT_ATTN", split == "all")
    g = load_golden(case)
    cshape, sshape, seeds = g["content_shape"], g["style_shape"], g["seeds"]
    c = seeded_image(*map(int, cshape), int(seeds[0])).to(DEV)
    s = seeded_image(*map(int, sshape), int(seeds[1])).to(DEV)
    fc, fs, fcs, cs = stylize(models(str(g["activation"]), torch.float32), c, s)
    cs = cs.cpu().numpy()
    assert mse01(cs, g["cs"]) < 1e-4
    assert mse_raw(cs, g["cs"]) < 1e-4
    if "fcs" in g:
        np.testing.assert_allclose(fcs.cpu().numpy(), g["fcs"], rtol=1e-3, atol=2e-3)
    for i in (0, 2):
        if f"fc{i}" in g:
            np.testing.assert_allclose(fc[i].cpu().numpy(), g[f"fc{i}"], rtol=1e-3, atol=1e-3)
            np.testing.assert_allclose(fs[i].cpu().numpy(), g[f"fs{i}"], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_forward_matches_numpy_oracle(dtype):
    from oracle import mhada_oracle as O
    ms = models("softmax", dtype)
    c = seeded_image(2, 128, 96, 31)
    s = seeded_image(2, 96, 128, 32)
    _, _, _, cs = stylize(ms, c.to(DEV), s.to(DEV))
    p = [O.to_numpy_params(m.state_dict()) for m in ms]
    _, _, _, ref = O.stylize(c.numpy(), s.numpy(), *p)
    assert mse01(cs.cpu().numpy(), ref) < 1e-4
    if dtype == torch.float32:
        assert mse_raw(cs.cpu().numpy(), ref) < 1e-4


def test_block_and_decoder_goldens():
    g = load_golden("block_b2_4x4_s3x5")
    blk = load_recipe(network.AdaAttnMultiHead(512, 8), "blk").to(DEV)
    with torch.no_grad():
        y = blk(*(torch.from_numpy(g[k]).to(DEV) for k in ("fc", "fs", "fcs")))
    np.testing.assert_allclose(y.cpu().numpy(), g["out"], rtol=1e-4, atol=1e-4)
    g = load_golden("decoder_b2_8x6")
    from mhada_hip.recipe import recipe_state_dict
    dec = network.Decoder()
    sd = recipe_state_dict("dec", {"decoder." + k: tuple(v.shape) for k, v in dec.state_dict().items()})
    dec.load_state_dict({k[len("decoder."):]: v for k, v in sd.items()}, strict=True)
    with torch.no_grad():
        y = dec.to(DEV)(torch.from_numpy(g["x"]).to(DEV))
    np.testing.assert_allclose(y.cpu().numpy(), g["y"], rtol=1e-4, atol=1e-4)


def test_api_shapes_and_calling_conventions():
    ms = models()
    c = seeded_image(2, 64, 64, 1).to(DEV)
    fc, fs, fcs, cs = stylize(ms, c, c)
    assert [tuple(t.shape) for t in fc] == [(2, 512, 8, 8)] * 3
    assert tuple(fcs.shape) == (2, 512, 8, 8) and tuple(cs.shape) == (2, 3, 64, 64)
    with torch.no_grad():
        fcs2, cs2 = ms[2]((fc, fs))  # the ptflops convention (adaDecoder.py:257-258)
    assert torch.equal(cs, cs2)
    # reference-style NCHW (non-view) inputs give the same result as the channels-last views
    with torch.no_grad():
        _, cs3 = ms[2]([t.contiguous() for t in fc], [t.contiguous() for t in fs])
    assert torch.equal(cs, cs3)


def test_feature_outputs_are_channels_last_nchw():
    """fc / fs / fcs are NCHW tensors in torch.channels_last memory format (views of the
    token-major storage; the reference's are contiguous NCHW, vit.py:165-166 / adaDecoder.py:205).
    Every torch op, .reshape and .contiguous() behave as on the reference's tensors; a raw
    .view(B, -1) needs .contiguous() first.  cs is contiguous NCHW."""
    ms = models()
    c = seeded_image(2, 64, 48, 1).to(DEV)
    fc, fs, fcs, cs = stylize(ms, c, c)
    assert cs.is_contiguous()
    for t in (*fc, *fs, fcs):
        assert t.is_contiguous(memory_format=torch.channels_last)
        ref = t.contiguous()
        assert torch.equal(t.reshape(2, -1), ref.view(2, -1))
        assert torch.equal(t.flatten(2).transpose(1, 2), ref.flatten(2).transpose(1, 2))
        assert torch.allclose(torch.nn.functional.avg_pool2d(t, 2), torch.nn.functional.avg_pool2d(ref, 2),
                              rtol=1e-6, atol=1e-5)
        with pytest.raises(RuntimeError):
            t.view(2, -1)


def test_bf16_autocast_selects_bf16_path():
    ms = models()
    for m in ms:
        m.compute_dtype = None  # an explicit compute_dtype takes precedence over autocast
    c = seeded_image(1, 64, 64, 5).to(DEV)
    with torch.no_grad():
        _, _, _, cs32 = stylize(ms, c, c)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, _, _, cs16 = stylize(ms, c, c)
    assert not torch.equal(cs32, cs16)
    assert mse01(cs32.cpu().numpy(), cs16.cpu().numpy()) < 1e-4


def test_vit_batch_one_reduces_to_value_projection():
    """At B=1 the batch-axis MHA is exactly out_proj(v_proj(x))."""
    import torch_ref
    vc = models()[0]
    x = seeded_image(1, 64, 64, 3).to(DEV)
    with torch.no_grad():
        ours = vc(x)
        ref = torch_ref.vit(x, {k: v for k, v in vc.state_dict().items()})
    for a, b in zip(ours, ref):
        assert ((a - b).norm() / b.norm()).item() < 1e-5


@pytest.mark.parametrize("res,B,dtype", [(512, 8, torch.float32), (1024, 4, torch.bfloat16)])
def test_full_size_against_torch_fp32(res, B, dtype):
    """BASELINE configs 2 and 3 at full size vs the fp32 PyTorch restatement on the device."""
    import torch_ref
    ms = models("softmax", dtype)
    c = seeded_image(B, res, res, 11 if res == 512 else 21).to(DEV)
    s = seeded_image(B, res, res, 12 if res == 512 else 22).to(DEV)
    _, _, _, cs = stylize(ms, c, s)
    sds = [{k: v.float() for k, v in m.state_dict().items()} for m in ms]
    with torch.no_grad():
        _, _, _, ref = torch_ref.stylize(c, s, *sds)
    a, b = cs.cpu().numpy(), ref.cpu().numpy()
    assert mse01(a, b) < 1e-4
    if dtype == torch.float32:
        assert mse_raw(a, b) < 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_graphed_stylizer_matches_eager(dtype):
    """mhada_hip.graphs.GraphedStylizer (one hipGraph replay of vit_c -> vit_s -> adaFormer ->
    clamp, infer_time.py:74-77) gives the eager call's bits, for new inputs on every replay."""
    from mhada_hip.graphs import GraphedStylizer
    ms = models(dtype=dtype)
    g = GraphedStylizer(*ms, (2, 3, 64, 96))
    for seed in (3, 5):
        c = seeded_image(2, 64, 96, seed).to(DEV)
        s = seeded_image(2, 64, 96, seed + 1).to(DEV)
        ref = stylize(ms, c, s)[3].clamp(0, 255)
        out = g(c, s)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    with pytest.raises(ValueError):
        g(torch.zeros(1, 3, 64, 96, device=DEV), torch.zeros(1, 3, 64, 96, device=DEV))
