"""Forward-path engine: the reference modules' forward passes expressed as sequences of
HIP launches on token-major ("NHWC") device buffers.

Layout in HBM (per forward call, B images, N = (H/8)(W/8) tokens, C = 512):
  * ViT residual stream       fp32 [B][N][C]            (LayerNorm inputs / residual adds)
  * GEMM operands             compute dtype (fp32 | bf16) [B*N][K]
  * per-layer ViT outputs     fp32 [B][N][C]; handed to callers as NCHW *views*
                              (x.view(B,h,w,C).permute(0,3,1,2)) — no transpose kernel
  * MHAda per block           Q [B][H][Nc][64], KV [B][H][Ns][128] (K | V'), and
                              VT [B][H][128][ceil64(Ns)] (V'^T | V'^2^T); out [B][Nc][C]
  * decoder                   NHWC activations in the compute dtype; the module output is
                              NCHW fp32 (B,3,8h,8w), written directly by the last conv.
Weights are repacked once per (dtype, parameter version) and cached on the module.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import weakref

import torch

from . import ops
from ._lib import ACT_COSINE, ACT_SOFTMAX

HEAD_DIM = 64
DECODER_LAYERS: Tuple[Tuple[str, bool], ...] = (
    # (name, upsample x2 applied to this layer's INPUT) — conv.py:78-94: bilinear x2 follows
    # conv1.0, conv1.4 and conv2.1, so conv1.1, conv2.0 and conv3.0 read an upsampled input.
    ("conv1.0", False), ("conv1.1", True), ("conv1.2", False), ("conv1.3", False),
    ("conv1.4", False), ("conv2.0", True), ("conv2.1", False), ("conv3.0", True),
)
LAST_LAYER = "conv3.1"
# Where the decoder's bilinear x2 runs: fused into the next conv's operand gather (4 taps per
# staged chunk, no extra HBM round trip) or as a standalone NHWC upsample kernel followed by a
# plain conv (one extra write+read of the upsampled tensor, but the conv keeps its lean
# gather and large tile).  Measured (tools/opbench.py conv): the standalone form is faster
# for every decoder layer in both dtypes (e.g. bf16 256->256 @256: 464 vs 903 us).
FUSE_UPSAMPLE = {torch.float32: False, torch.bfloat16: False}


def _fuse_upsample(dt: torch.dtype, w: torch.Tensor) -> bool:
    """The bf16 64 -> 64 layer runs on the direct tile kernel (csrc/conv_tile.hip), whose fused
    upsample is bit-identical to the separate one and 13 % faster (523 vs 600 us at 1024^2 B4)."""
    return FUSE_UPSAMPLE[dt] or (dt == torch.bfloat16 and w.shape[0] == 64 and w.shape[1] == 9 * 64)


# ---------------------------------------------------------------------------------------
# optional per-kernel event timing (bench.py): HIP events recorded on the launch stream
# ---------------------------------------------------------------------------------------
_event_log = None  # dict name -> list of (start, end) torch.cuda.Event, or None (off)


def record_kernel_events(log) -> None:
    """Enable (pass a dict) or disable (None) event brackets around the named launches."""
    global _event_log
    _event_log = log


class _timed:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if _event_log is not None:
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *exc):
        if _event_log is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _event_log.setdefault(self.name, []).append((self.s, e))
        return False


# ---------------------------------------------------------------------------------------
# compute dtype & weight caches
# ---------------------------------------------------------------------------------------
def resolve_compute_dtype(module: torch.nn.Module) -> torch.dtype:
    """fp32 by default (the reference's arithmetic); bf16 when the module's
    ``compute_dtype`` says so or a CUDA autocast region asks for a 16-bit dtype (the HIP path
    has bf16 MFMA kernels only, so float16 autocast also runs bf16)."""
    explicit = getattr(module, "compute_dtype", None)
    if explicit is not None:
        if explicit not in (torch.float32, torch.bfloat16):
            raise ValueError(f"compute_dtype must be torch.float32 or torch.bfloat16, got {explicit}")
        return explicit
    if torch.is_autocast_enabled("cuda"):
        if torch.get_autocast_dtype("cuda") in (torch.bfloat16, torch.float16):
            return torch.bfloat16
    return torch.float32


def _signature(module: torch.nn.Module):
    return tuple((p.data_ptr(), p._version) for p in module.parameters())


def cached_prep(module: torch.nn.Module, dtype: torch.dtype, build):
    cache: Dict = module.__dict__.setdefault("_mhada_prep", {})
    key = (dtype, _signature(module))
    hit = cache.get(dtype)
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        prep = build(dtype)
    cache[dtype] = (key, prep)
    return prep


def require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the MI355X-native network runs on ROCm device tensors only; "
                           "move the module and inputs with .to('cuda')")


def to_tokens(x: torch.Tensor) -> torch.Tensor:
    """NCHW (any strides) -> contiguous fp32 [B][H][W][C] (zero-copy for this package's own
    channels-last views)."""
    t = x.permute(0, 2, 3, 1)
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def tokens_to_nchw(t: torch.Tensor, h: int, w: int) -> torch.Tensor:
    B, _, C = t.shape
    return t.view(B, h, w, C).permute(0, 3, 1, 2)


# ---------------------------------------------------------------------------------------
# ViT (network/vit.py)
# ---------------------------------------------------------------------------------------
def vit_prep(vit, dtype):
    def build(dt):
        pe = vit.patch_embedding.conv_proj
        layers = []
        for blk in vit.encoder:
            att = blk.attention
            layers.append(dict(
                ln1_g=blk.ln1.weight.float().contiguous(), ln1_b=blk.ln1.bias.float().contiguous(),
                ln2_g=blk.ln2.weight.float().contiguous(), ln2_b=blk.ln2.bias.float().contiguous(),
                w_qkv=att.in_proj_weight.to(dt).contiguous(), b_qkv=att.in_proj_bias.float().contiguous(),
                w_o=att.out_proj.weight.to(dt).contiguous(), b_o=att.out_proj.bias.float().contiguous(),
                w1=blk.mlp[0].weight.to(dt).contiguous(), b1=blk.mlp[0].bias.float().contiguous(),
                w2=blk.mlp[2].weight.to(dt).contiguous(), b2=blk.mlp[2].bias.float().contiguous(),
                heads=att.num_heads, eps=blk.ln1.eps))
        return dict(patch_w=pe.weight.reshape(pe.weight.shape[0], -1).to(dt).contiguous(),
                    patch_b=pe.bias.float().contiguous(), layers=layers, pos={})
    return cached_prep(vit, dtype, build)


_NUM_CUS: Dict = {}


def _split3_fills(M: int, N: int, dev: torch.device) -> bool:
    """ops.F32_SPLIT and the SPLIT3 GEMM's 256x256 tiles cover >= 7/8 of the CUs (the rule the fp32
    GEMM dispatch uses for its own persistent kernel)."""
    if not ops.F32_SPLIT:
        return False
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _NUM_CUS:
        _NUM_CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return 8 * ((M + 255) // 256) * ((N + 255) // 256) >= 7 * _NUM_CUS[idx]


def _w6(L: dict, key: str) -> torch.Tensor:
    """The SPLIT3 form of an fp32 ViT weight (ops.split3_weight), built once per prepared layer."""
    k6 = key + "_split3"
    if k6 not in L:
        with torch.no_grad():
            L[k6] = ops.split3_weight(L[key])
    return L[k6]


def vit_forward(vit, x: torch.Tensor) -> List[torch.Tensor]:
    """VisionTransformer.forward (vit.py:148-169) on the HIP path."""
    require_device(x, "VisionTransformer")
    dt = resolve_compute_dtype(vit)
    prep = vit_prep(vit, dt)
    if x.dim() != 4 or x.shape[1] != 3:
        raise ValueError(f"expected an image batch (B, 3, H, W), got {tuple(x.shape)}")
    img = x.float().contiguous()
    B, _, H, W = img.shape
    p = vit.patch_size
    h, w = H // p, W // p
    N = h * w
    C = prep["patch_w"].shape[0]
    pos = None
    if vit.pos_embedding is not None:
        pos = prep["pos"].get((h, w))
        if pos is None:
            pos = ops.pos_embed(vit.pos_embedding.pos_embed.detach().float().contiguous(), h, w)
            prep["pos"][(h, w)] = pos
    tok = ops.patch_embed(img, prep["patch_w"], prep["patch_b"], pos, p)  # [B][N][C] fp32
    xs = tok.view(B * N, C)
    outs = []
    for L in prep["layers"]:
        # fp32: LayerNorm -> bf16 planes -> SPLIT3 GEMM (fp32-accurate on the bf16 MFMA) where the
        # 256x256 tiles fill the chip; small batches keep the fp32 MFMA GEMMs (their 128x128 tiles
        # cover more CUs than 6x-longer SPLIT3 tiles would)
        split = dt == torch.float32 and _split3_fills(B * N, 3 * C, xs.device)
        split_mlp = dt == torch.float32 and _split3_fills(B * N, C, xs.device)
        if split:
            qkv = ops.linear_split3(ops.layernorm_split3(xs, L["ln1_g"], L["ln1_b"], L["eps"]), _w6(L, "w_qkv"),
                                    L["b_qkv"], dt)
        else:
            hb = ops.layernorm(xs, L["ln1_g"], L["ln1_b"], dt, L["eps"])
            qkv = ops.linear(hb, L["w_qkv"], L["b_qkv"], dt)
        att = ops.vit_batch_attn(qkv.view(B, N, 3 * C), B, N, L["heads"])
        xs = ops.linear(att.view(B * N, C), L["w_o"], L["b_o"], torch.float32, residual=xs)
        if split_mlp:  # MLP1 writes its ReLU output as planes, MLP2 consumes them (SPLIT3 both)
            m1 = ops.linear_split3(ops.layernorm_split3(xs, L["ln2_g"], L["ln2_b"], L["eps"]), _w6(L, "w1"),
                                   L["b1"], dt, relu=True, out_planes=True)
            xs = ops.linear_split3(m1, _w6(L, "w2"), L["b2"], torch.float32, residual=xs)
        else:
            h2 = ops.layernorm(xs, L["ln2_g"], L["ln2_b"], dt, L["eps"])
            m1 = ops.linear(h2, L["w1"], L["b1"], dt, relu=True)
            xs = ops.linear(m1, L["w2"], L["b2"], torch.float32, residual=xs)
        outs.append(tokens_to_nchw(xs.view(B, N, C), h, w))
    return outs


# ---------------------------------------------------------------------------------------
# MHAda blocks (network/adaDecoder.py)
# ---------------------------------------------------------------------------------------
def block_prep(blk, dtype):
    def build(dt):
        H = blk.num_heads
        d = blk.head_dim

        def stack(lst):
            return torch.stack([m.weight.reshape(d, d) for m in lst]).float().contiguous()

        def stackb(lst):
            return torch.stack([m.bias for m in lst]).float().contiguous()
        C = H * d
        return dict(wf=stack(blk.f_list), wg=stack(blk.g_list), wh=stack(blk.h_list),
                    bf=stackb(blk.f_list), bg=stackb(blk.g_list), bh=stackb(blk.h_list),
                    w_out=blk.out_conv.weight.reshape(C, C).to(dt).contiguous(),
                    b_out=blk.out_conv.bias.float().contiguous())
    return cached_prep(blk, dtype, build)


class _Feat:
    """A token-major fp32 feature map with lazily computed InstanceNorm statistics."""

    def __init__(self, t: torch.Tensor, h: int, w: int):
        self.t, self.h, self.w = t, h, w  # t: [B][N][C]
        self._stats = None
        self.t16 = None  # optional bf16 copy of t (written by the producing GEMM)

    @classmethod
    def from_nchw(cls, x: torch.Tensor):
        _, _, h, w = x.shape
        t = to_tokens(x)
        return cls(t.view(t.shape[0], h * w, t.shape[3]), h, w)

    def stats(self):
        if self._stats is None:
            self._stats = ops.instnorm_stats(self.t)
        return self._stats


def block_forward(blk, fc: _Feat, fs: Optional[_Feat], fcs: _Feat, dt: torch.dtype,
                  side: Optional[dict] = None, want_bf16: bool = False) -> _Feat:
    """AdaAttnMultiHead.forward (adaDecoder.py:162-206).

    ``side`` carries the block's style-only tensors (IN statistics of fs, the K|V' projection and
    its V'^T image): when it is filled they are reused (fs may then be None), when it is an empty
    dict they are computed and stored into it (the per-style cache of adaformer_forward).
    ``want_bf16``: the out_conv GEMM also writes a bf16 copy of the block output (``.t16``) for
    the decoder's first conv (the last block of a bf16 forward)."""
    if blk.head_dim != HEAD_DIM:
        raise ValueError(f"the HIP MHAda kernels implement head_dim={HEAD_DIM} (qkv_dim/num_heads), "
                         f"got {blk.head_dim}")
    prep = block_prep(blk, dt)
    H = blk.num_heads
    C = H * HEAD_DIM
    B, Nc, Cc = fc.t.shape
    cached = bool(side)
    mom = img = kv = vt = None
    act = ACT_COSINE if blk.activation_name == "cosine" else ACT_SOFTMAX
    # fp32 softmax: the SPLIT3 attention on bf16 planes of K and V'^T | V'^2^T (csrc/attn_split3.hip)
    split_attn = act == ACT_SOFTMAX and dt == torch.float32 and ops.F32_SPLIT_ATTN
    if cached:
        mu_s, rstd_s, mom, Ns = side["mu_s"], side["rstd_s"], side.get("mom"), side["Ns"]
        kv, vt, img = side.get("kv"), side.get("vt"), side.get("img")
        if side["B"] != B:
            raise ValueError(f"cached style batch {side['B']} != content batch {B}")
    else:
        if fs.t.shape[2] != C:
            raise ValueError(f"channel mismatch: block expects {C}")
        mu_s, rstd_s = fs.stats()
    if Cc != C or fcs.t.shape[2] != C:
        raise ValueError(f"channel mismatch: block expects {C}")
    mu_c, rstd_c = fc.stats()
    mu_o, rstd_o = fcs.stats()
    wq, wkv, bkv, v_mu = ops.fold_block(prep["wf"], prep["wg"], prep["wh"], prep["bg"], prep["bh"],
                                        rstd_c, mu_s, rstd_s, dt, ops.LOG2E if act == ACT_SOFTMAX else 1.0)
    dev = fc.t.device
    q = torch.empty(B, H, Nc, HEAD_DIM, device=dev, dtype=dt)
    ops.gemm(a=fc.t, w=wq, c=q, M=Nc, N=HEAD_DIM, K=HEAD_DIM, compute=dt, lda=C, sa=(Nc * C, HEAD_DIM),
             nb=(B, H), a_mu=mu_c, smu=(C, HEAD_DIM), ldw=HEAD_DIM, sw=(H * HEAD_DIM * HEAD_DIM, HEAD_DIM * HEAD_DIM),
             bias=prep["bf"], sb=(0, HEAD_DIM), ldc=HEAD_DIM, sc=(H * Nc * HEAD_DIM, Nc * HEAD_DIM))
    if not cached and split_attn:
        Ns = fs.t.shape[1]
        # K|V' projection written straight as the SPLIT3 attention's bf16 plane image (no fp32 kv / vt)
        img = ops.kv_proj_split3(fs.t, mu_s, wkv, bkv)
        if side is not None:
            side.update(mu_s=mu_s, rstd_s=rstd_s, img=img, Ns=Ns, B=B)
    elif not cached:
        Ns = fs.t.shape[1]
        # K|V' projection: K rows into kv[..., :64] (the attention's K operand), V' straight into
        # the transposed V'^T | V'^2^T image vt (the GEMM's vt epilogue; kv[..., 64:] unused)
        kv = torch.empty(B, H, Ns, 2 * HEAD_DIM, device=dev, dtype=dt)
        ldt = (Ns + 63) // 64 * 64
        vt = torch.empty(B, H, 2 * HEAD_DIM, ldt, device=dev, dtype=dt)
        ops.gemm(a=fs.t, w=wkv, c=kv, M=Ns, N=2 * HEAD_DIM, K=HEAD_DIM, compute=dt, lda=C, sa=(Ns * C, HEAD_DIM),
                 nb=(B, H), a_mu=mu_s, smu=(C, HEAD_DIM), ldw=HEAD_DIM,
                 sw=(H * 2 * HEAD_DIM * HEAD_DIM, 2 * HEAD_DIM * HEAD_DIM), bias=bkv, sb=(0, 2 * HEAD_DIM),
                 ldc=2 * HEAD_DIM, sc=(H * Ns * 2 * HEAD_DIM, Ns * 2 * HEAD_DIM),
                 vt=vt, ldt=ldt, svt=(H * 2 * HEAD_DIM * ldt, 2 * HEAD_DIM * ldt))
        if act == ACT_COSINE:
            # the cosine activation's linear form: the style-side moments replace the Nc x Ns loop
            ops.cosine_prep(None, kv)
            mom = ops.cosine_moments(kv, vt)
        if side is not None:
            side.update(mu_s=mu_s, rstd_s=rstd_s, kv=kv, vt=vt, mom=mom, Ns=Ns, B=B)
    if act == ACT_COSINE:
        ops.cosine_prep(q, None)
        with _timed("mhada_attn"):
            att = ops.cosine_attn(q, mom, fcs.t, mu_o, rstd_o, v_mu)  # [B][Nc][C] dt
    elif split_attn:
        with _timed("mhada_attn"):
            att = ops.attn_split3(q, img, Ns, fcs.t, mu_o, rstd_o, v_mu)  # [B][Nc][C] fp32
    else:
        with _timed("mhada_attn"):
            att = ops.mhada_attn(q, kv, vt, fcs.t, mu_o, rstd_o, v_mu, act)  # [B][Nc][C] dt
    out = torch.empty(B * Nc, C, device=dev, dtype=torch.float32)
    t16 = torch.empty(B * Nc, C, device=dev, dtype=torch.bfloat16) if want_bf16 else None
    ops.gemm(a=att.view(B * Nc, C), w=prep["w_out"], c=out, M=B * Nc, N=C, K=C, compute=dt, lda=C, ldw=C,
             bias=prep["b_out"], ldc=C, c2=t16, ldc2=C)
    f = _Feat(out.view(B, Nc, C), fc.h, fc.w)
    f.t16 = None if t16 is None else t16.view(B, Nc, C)
    return f


def style_cache(ada, fs: Sequence[torch.Tensor], dt: torch.dtype):
    """Per-style cache of the blocks' style-side tensors (the video path of
    infer_video.py:58-92: fs = vit_s(style) once, adaFormer(fc, fs) per frame).

    A hit needs the SAME fs tensor objects (held by weak reference, so a freed and reallocated
    buffer can never alias), unchanged in place (tensor._version), the same compute dtype and
    unchanged block parameters.  Returns (per-block dicts, hit).  ``ada.cache_style = False``
    turns the cache off."""
    if not getattr(ada, "cache_style", True):
        return [None] * len(ada.adaAttnHead), False
    sig = tuple(_signature(b) for b in ada.adaAttnHead)
    vers = tuple(t._version for t in fs)
    mode = (dt, ops.F32_SPLIT_ATTN)  # the cached side tensors depend on the attention form
    c = ada.__dict__.get("_mhada_style")
    if (c is not None and c["mode"] == mode and c["sig"] == sig and c["vers"] == vers
            and len(c["refs"]) == len(fs) and all(r() is t for r, t in zip(c["refs"], fs))):
        return c["sides"], True
    sides = [dict() for _ in ada.adaAttnHead]
    ada.__dict__["_mhada_style"] = dict(mode=mode, sig=sig, vers=vers, refs=[weakref.ref(t) for t in fs], sides=sides)
    return sides, False


# ---------------------------------------------------------------------------------------
# Decoder (network/conv.py)
# ---------------------------------------------------------------------------------------
def decoder_prep(dec, dtype):
    def build(dt):
        mods = dict(dec.named_modules())
        layers = []
        for name, up in DECODER_LAYERS:
            conv = mods[name].conv.conv
            w = conv.weight.permute(0, 2, 3, 1).reshape(conv.weight.shape[0], -1).to(dt).contiguous()
            # fp32: the Winograd-transformed filters (ops.conv3x3 runs F(2x2,3x3) when eligible)
            u = ops.wino_weights(w) if dt == torch.float32 and w.shape[0] % 64 == 0 and (w.shape[1] // 9) % 8 == 0 \
                else None
            layers.append((w, conv.bias.float().contiguous(), up, u))
        last = mods[LAST_LAYER].conv.conv
        # [out][cin][ky][kx] -> [ky*3+kx][cin][out]
        return dict(layers=layers, w_last=last.weight.permute(2, 3, 1, 0).float().contiguous(),
                    b_last=last.bias.float().contiguous())
    return cached_prep(dec, dtype, build)


def decoder_forward_tokens(dec, x_nhwc: torch.Tensor, dt: torch.dtype, clamp255: bool = False,
                           x16: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decoder.forward (conv.py:96-100) on NHWC input; returns NCHW fp32 (B,3,8h,8w).  ``x16``: a
    bf16 copy of the input (bf16 compute: the first conv then runs on the bf16 ping-pong GEMM
    instead of converting fp32 rows on load)."""
    prep = decoder_prep(dec, dt)
    x = x16 if (x16 is not None and dt == torch.bfloat16) else x_nhwc
    for w, b, up, u in prep["layers"]:
        if up and not _fuse_upsample(dt, w):
            x = ops.upsample2x(x)
            up = False
        x = ops.conv3x3(x, w, b, dt, upsample=up, relu=True, wino_u=u)
    return ops.conv3x3_out3(x, prep["w_last"], prep["b_last"], clamp255=clamp255)


def adaformer_forward(ada, fc: Sequence[torch.Tensor], fs: Sequence[torch.Tensor]):
    """AdaAttnTransformerMultiHead.forward (adaDecoder.py:253-268): returns (fcs, cs)."""
    require_device(fc[0], "AdaAttnTransformerMultiHead")
    dt = resolve_compute_dtype(ada)
    L = ada.num_layers
    fcf = [_Feat.from_nchw(t) for t in fc[:L]]
    sides, hit = style_cache(ada, fs[:L], dt)
    fsf = [None] * L if hit else [_Feat.from_nchw(t) for t in fs[:L]]
    fcs = fcf[0]
    for i in range(L):
        fcs = block_forward(ada.adaAttnHead[2 * i], fcf[i], fsf[i], fcs, dt, sides[2 * i])
        fcs = block_forward(ada.adaAttnHead[2 * i + 1], fcs, fsf[i], fcs, dt, sides[2 * i + 1],
                            want_bf16=(dt == torch.bfloat16 and i == L - 1))
    B, N, C = fcs.t.shape
    x16 = None if fcs.t16 is None else fcs.t16.view(B, fcs.h, fcs.w, C)
    cs = decoder_forward_tokens(ada.decoder, fcs.t.view(B, fcs.h, fcs.w, C), dt, x16=x16)
    return tokens_to_nchw(fcs.t, fcs.h, fcs.w), cs
