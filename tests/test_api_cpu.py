"""Host-side checks of the drop-in network/ API and the C-ABI library (no GPU needed)."""
import json
import os
import re

import pytest
import torch

import network
from mhada_hip import _lib
from mhada_hip.recipe import load_recipe
from conftest import GOLDEN, REPO


def _keys():
    with open(os.path.join(GOLDEN, "state_dict_keys.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name,ctor", [
    ("vit_c", lambda: network.VisionTransformer(pos_embedding=True)),
    ("vit_s", lambda: network.VisionTransformer(pos_embedding=False)),
    ("ada", lambda: network.AdaAttnTransformerMultiHead()),
    ("block_512_8", lambda: network.AdaAttnMultiHead(512, 8)),
    ("decoder", lambda: network.Decoder()),
])
def test_state_dict_keys_match_reference(name, ctor):
    ref = _keys()[name]
    mine = {k: list(v.shape) for k, v in ctor().state_dict().items()}
    assert mine == ref


def test_reference_checkpoint_roundtrip(tmp_path):
    """A reference-format checkpoint (torch.save(state_dict)) loads strictly, weights_only."""
    vit = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c")
    path = tmp_path / "ViT_C.pth"
    torch.save(vit.state_dict(), path)
    vit2 = network.VisionTransformer(pos_embedding=True)
    vit2.load_state_dict(torch.load(path, weights_only=True), strict=True)
    for k, v in vit.state_dict().items():
        assert torch.equal(v, vit2.state_dict()[k])


def test_constructor_errors_mirror_reference():
    with pytest.raises(ValueError):
        network.AdaAttnMultiHead(512, 7)           # adaDecoder.py:137-138
    with pytest.raises(ValueError):
        network.AdaAttnTransformerMultiHead(activation="relu")  # adaDecoder.py:160
    with pytest.raises(ValueError):
        network.AdaAttnForLoss(256, 448, activation="tanh")      # adaDecoder.py:50
    network.AdaAttnTransformerMultiHead(activation="cosine")


def test_cpu_tensors_take_the_aten_form_not_the_engine(monkeypatch):
    """infer_image.py:48 picks "cpu" when no GPU is present: CPU tensors run the aten form of the
    reference expression (autograd_path), never the HIP engine (whose launches would need device
    pointers).  Device tensors are the only ones the engine sees."""
    from mhada_hip import engine

    def boom(*a, **k):
        raise AssertionError("the HIP engine must not be called with CPU tensors")
    for name in ("vit_forward", "adaformer_forward", "block_forward", "decoder_forward_tokens"):
        monkeypatch.setattr(engine, name, boom)
    vit = network.VisionTransformer()
    ada = network.AdaAttnTransformerMultiHead()
    with torch.no_grad():
        f = vit(torch.rand(1, 3, 64, 64) * 255)
        fcs, cs = ada(f, f)
        blk = ada.adaAttnHead[0](f[0], f[0], f[0])
    assert cs.shape == (1, 3, 64, 64) and torch.isfinite(cs).all()
    assert blk.shape == (1, 512, 8, 8) and torch.isfinite(blk).all()


def test_compute_dtype_resolution():
    from mhada_hip import engine
    m = network.VisionTransformer()
    assert engine.resolve_compute_dtype(m) == torch.float32
    m.compute_dtype = torch.bfloat16
    assert engine.resolve_compute_dtype(m) == torch.bfloat16
    m.compute_dtype = torch.float16
    with pytest.raises(ValueError):
        engine.resolve_compute_dtype(m)


def _header_symbols():
    with open(os.path.join(REPO, "include", "mhada_hip.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|long long|const char\*)\s+(mhada_\w+)\s*\(", src, re.M)))


def test_library_loads_and_exports_every_header_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmhada_hip.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes signatures must cover the header exactly"
    assert lib.mhada_abi_version() == _lib.ABI_VERSION


def test_tuning_table_read_once_and_settable():
    """Kernel-variant knobs: read once at library init, changed only through mhada_set_tuning."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmhada_hip.so not built")
    assert _lib.get_tuning("attn_fixed_shift") == 1
    with _lib.tuning(attn_fixed_shift=0, attn_tk=64):
        assert _lib.get_tuning("attn_fixed_shift") == 0 and _lib.get_tuning("attn_tk") == 64
        os.environ["MHADA_ATTN_FIXED_SHIFT"] = "1"  # the environment is not re-read per call
        try:
            assert _lib.get_tuning("attn_fixed_shift") == 0
        finally:
            del os.environ["MHADA_ATTN_FIXED_SHIFT"]
    assert _lib.get_tuning("attn_fixed_shift") == 1 and _lib.get_tuning("attn_tk") == 128
    with pytest.raises(ValueError):
        _lib.set_tuning("no_such_knob", 1)
    with pytest.raises(ValueError):
        _lib.set_tuning("attn_tk", 96)


def test_abi_argument_errors_without_gpu():
    """Argument validation happens on the host before any launch."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmhada_hip.so not built")
    lib = _lib.load()
    assert lib.mhada_layernorm(None, None, 0, None, None, 4, 512, 1e-6, None) == 1
    assert b"bad args" in lib.mhada_last_error()
    args = _lib.GemmArgs()
    args.M, args.N, args.K, args.nb1, args.nb2 = 4, 4, 4, 1, 1
    args.compute = 7
    assert lib.mhada_gemm(args, None) == 1
    assert b"compute" in lib.mhada_last_error()
    assert lib.mhada_attn(*([None] * 8), 0, 1, 8, 64, 64, 0, None) == 1


def test_wino_eligible_respects_32bit_offsets():
    """shapes past the Winograd kernel's 32-bit element offsets fall back to the
    implicit-GEMM conv instead of raising (meta tensors: no memory, no GPU)."""
    from mhada_hip import ops
    w = torch.empty(64, 9 * 64, dtype=torch.float32, device="meta")
    assert ops.wino_eligible(torch.empty(8, 512, 512, 64, device="meta"), w, False)
    assert not ops.wino_eligible(torch.empty(8, 2048, 2048, 64, device="meta"), w, False)


def test_ds_spill_rule_is_shape_only(monkeypatch):
    """the attention backward's spill / recompute choice never looks at free device
    memory (that made dQ's bits depend on allocator state)."""
    from mhada_hip import ops

    def boom(*a, **k):
        raise AssertionError("the path rule must not query device memory")
    monkeypatch.setattr(torch.cuda, "mem_get_info", boom)
    assert ops.ds_spill_eligible(3 * 8 * 8, 4096, 4096)  # 512^2 B8, three AdaFormer calls batched
    assert not ops.ds_spill_eligible(4, 4096, 4094)       # Ns % 4 != 0
    assert not ops.ds_spill_eligible(1024, 8192, 8192)    # past DS_SPILL_BYTES


def test_vgg19_loads_torchvision_feature_weights(tmp_path):
    """real VGG19 weights from a local torchvision checkpoint (features.{i}.*
    keys, classifier ignored) load into the slices; a missing conv raises."""
    import torch
    vgg = network.VGG19()
    g = torch.Generator().manual_seed(3)
    tv = {}
    for name, p in vgg.named_parameters():
        s, i, t = name.split(".")
        tv[f"features.{i}.{t}"] = torch.randn(p.shape, generator=g)
    tv["classifier.0.weight"] = torch.randn(4096, 25088 // 64, generator=g)  # ignored
    torch.save(tv, tmp_path / "vgg19-dcbb9e9d.pth")
    vgg.load_torchvision_features(str(tmp_path / "vgg19-dcbb9e9d.pth"))
    for name, p in vgg.named_parameters():
        s, i, t = name.split(".")
        assert torch.equal(p, tv[f"features.{i}.{t}"])
        assert not p.requires_grad
    del tv["features.28.bias"]
    with pytest.raises(KeyError):
        network.VGG19().load_torchvision_features(tv)
