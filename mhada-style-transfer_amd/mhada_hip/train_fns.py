"""Autograd Functions of the training path on the HIP kernels (fp32, NHWC activations).

Each Function takes the reference module's own parameter tensors (``nn.Conv2d.weight`` /
``.bias``), so autograd delivers gradients to exactly the parameters whose state_dict keys match
the reference, and runs its forward and backward through libmhada_hip.so:

* ``conv3x3``  — ReflectionPad2d(1) + Conv2d 3x3 (+ReLU) of the decoder (conv.py:23-45) or the
  zero-padded Conv2d(padding=1) (+ReLU) of VGG19 (vgg19.py slices, torchvision cfg E).
  forward: the implicit-GEMM conv (mhada_gemm, CONV3X3 / CONV3X3_ZERO, bias+ReLU epilogue);
  backward: ReLU mask (mhada_relu_bwd), input gradient = the conv of dY with the flipped,
  transposed weights (zero pad 1, or the full correlation + mhada_reflect_fold for the reflect
  pad), weight gradient = mhada_gemm_tn over the im2col of the input, bias = the column sums of
  dY from the same mhada_gemm_tn pass.
* ``linear`` — nn.Linear / the 1x1 out_conv on token rows (vit.py:49-63 MHA projections and MLP,
  adaDecoder.py:152,205), optional fused ReLU: forward mhada_gemm; backward dX = dY W (mhada_gemm
  with W^T), dW = dY^T X and db = colsum(dY) in one mhada_gemm_tn pass.
* ``patch_embed`` — the 8x8 / stride-8 patch conv (vit.py:105-117): forward mhada_gemm PATCH8,
  weight gradient mhada_gemm_tn PATCH8 (the input image needs no gradient in training).
* ``maxpool2``, ``upsample2x`` (conv.py:71), ``vgg_input`` (vgg19.py:6-12) and their adjoints.
"""
from __future__ import annotations

import weakref
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from . import ops
from ._lib import A_CONV3X3, A_CONV3X3_ZERO, A_PATCH8, A_ROWS

F32 = torch.float32


def _ceil(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def _pack_fwd(weight: torch.Tensor, cx: int) -> torch.Tensor:
    """(Co, Ci, 3, 3) -> [Co][9*cx] with k = tap*cx + ci (channels ci >= Ci zero)."""
    co, ci = weight.shape[:2]
    w = weight.detach().permute(0, 2, 3, 1)
    if cx != ci:
        w = F.pad(w, (0, cx - ci))
    return w.reshape(co, 9 * cx).contiguous()


def _pack_dgrad(weight: torch.Tensor, cx: int, cg: int) -> torch.Tensor:
    """W'[ci][ky][kx][co] = W[co][ci][2-ky][2-kx] -> [cx][9*cg] (ci >= Ci rows and co >= Co
    columns zero): the weights of the conv that computes the input gradient."""
    co, ci = weight.shape[:2]
    w = weight.detach().flip(2, 3).permute(1, 2, 3, 0)  # (Ci, 3, 3, Co)
    w = F.pad(w, (0, cg - co, 0, 0, 0, 0, 0, cx - ci))
    return w.reshape(cx, 9 * cg).contiguous()


# Packed / Winograd-transformed copies of frozen weights (VGG19), keyed by the weight tensor's
# identity and checked against its version counter.  Held here, not on the Parameter: pickling,
# deepcopy or torch.save(module) of the VGG then carry no extra GPU copies.  An entry dies with
# its weight (weakref.finalize), and a recycled id() can never alias (the entry holds a weakref
# whose referent is compared by identity).
_PACK_CACHE: Dict[int, tuple] = {}


def _pack_slot(weight: torch.Tensor) -> Dict:
    key = id(weight)
    ent = _PACK_CACHE.get(key)
    if ent is None or ent[0]() is not weight:
        ent = (weakref.ref(weight), {})
        _PACK_CACHE[key] = ent
        weakref.finalize(weight, _PACK_CACHE.pop, key, None)
    return ent[1]


def _cached(weight: torch.Tensor, kind: str, *dims) -> torch.Tensor:
    """Packed weights of a frozen layer (VGG19), cached per weight tensor and keyed by its
    version counter; trainable weights change every step and are packed per call."""
    if weight.requires_grad:
        return _pack_fwd(weight, *dims) if kind == "f" else _pack_dgrad(weight, *dims)
    cache = _pack_slot(weight)
    key = (kind,) + dims
    hit = cache.get(key)
    if hit is not None and hit[0] == weight._version:
        return hit[1]
    w = _pack_fwd(weight, *dims) if kind == "f" else _pack_dgrad(weight, *dims)
    cache[key] = (weight._version, w)
    return w


def _wino(weight: torch.Tensor, kind: str, packed: torch.Tensor, *dims) -> Optional[torch.Tensor]:
    """Winograd-transformed filters of a frozen layer's packed weights (cached like _cached);
    None for trainable weights (ops.conv3x3 transforms them per call) or ineligible shapes."""
    if weight.requires_grad or packed.dtype != F32 or packed.shape[0] % 64 or (packed.shape[1] // 9) % 8:
        return None
    cache = _pack_slot(weight)
    key = ("u", kind) + dims
    hit = cache.get(key)
    if hit is not None and hit[0] == weight._version:
        return hit[1]
    u = ops.wino_weights(packed)
    cache[key] = (weight._version, u)
    return u


class Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, pad_mode: str, relu: bool,
                grad_masked: bool = False, relu_input: bool = False):
        if x.dtype != F32 or not x.is_contiguous():
            raise ValueError("conv3x3 (training) takes contiguous fp32 NHWC activations")
        B, H, W, cx = x.shape
        co, ci = weight.shape[:2]
        if ci > cx or cx % 32:
            raise ValueError(f"conv3x3: input channels {cx} must be a multiple of 32 and >= {ci}")
        ldc = _ceil(co, 4)
        y = (torch.zeros if ldc != co else torch.empty)(B, H, W, ldc, device=x.device, dtype=F32)
        wf = _cached(weight, "f", cx)
        ops.conv3x3(x, wf, bias.detach().float().contiguous(), F32, upsample=False,
                    relu=relu, pad_mode=pad_mode, pad=1, out=y, wino_u=_wino(weight, "f", wf, cx))
        ctx.save_for_backward(x, weight, y)
        # grad_masked: the output's only consumer (MaxPool2Fn(relu_input=True)) hands back the
        # gradient with the ReLU adjoint already applied
        # relu_input: x is the ReLU output of a Conv3x3Fn(grad_masked=True) whose only consumer is this
        # conv: the input gradient leaves with that ReLU's adjoint applied (the Winograd dgrad's output
        # stage / the reflect fold zero it where x <= 0), so the producer skips its relu_bwd pass
        ctx.pad_mode, ctx.relu, ctx.grad_masked, ctx.relu_input = pad_mode, relu, grad_masked, relu_input
        return y if ldc == co else y[..., :co].contiguous()

    @staticmethod
    def backward(ctx, gy: torch.Tensor):
        x, weight, y = ctx.saved_tensors
        B, H, W, cx = x.shape
        co = weight.shape[0]
        ldc = y.shape[-1]
        gy = gy.contiguous()
        if ldc != co:
            gy = F.pad(gy, (0, ldc - co))
        g = ops.relu_bwd(gy, y) if ctx.relu and not ctx.grad_masked else gy
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            cg = _ceil(co, 32)
            gk = g if cg == ldc else F.pad(g, (0, cg - ldc))
            wt = _cached(weight, "d", cx, cg)
            ut = _wino(weight, "d", wt, cx, cg)
            mask = x if ctx.relu_input else None
            if ctx.pad_mode == "zero":
                gx = ops.conv3x3(gk, wt, None, F32, upsample=False, relu=False, pad_mode="zero", pad=1, wino_u=ut,
                                 relu_mask=mask)
            else:
                gx = ops.reflect_fold(ops.conv3x3(gk, wt, None, F32, upsample=False, relu=False, pad_mode="zero",
                                                  pad=2, wino_u=ut), relu_mask=mask)
        if ctx.needs_input_grad[1] and ops.wgrad_wino_eligible(x, g, co):
            # Winograd F(2x2,3x3) weight gradient (2.25x fewer products than the im2col TN GEMM),
            # bias gradient from its dY transform
            dw, cs = ops.conv3x3_wgrad_wino(x, g, co, ctx.pad_mode, bias=ctx.needs_input_grad[2])
            gw = dw.view(co, 3, 3, cx)[:, :, :, :weight.shape[1]].permute(0, 3, 1, 2).contiguous()
            if ctx.needs_input_grad[2]:
                gb = cs
        elif ctx.needs_input_grad[1]:
            mode = A_CONV3X3 if ctx.pad_mode == "reflect" else A_CONV3X3_ZERO
            # M = ldc (the zero-padded channel columns of g) keeps the vectorised A loads; the bias
            # gradient (column sums of g) comes out of the same pass
            dw, cs = ops.gemm_tn(g, x, M=ldc, N=9 * cx, K=B * H * W, lda=ldc, b_mode=mode, img=(cx, H, W), pad=1,
                                 colsum=True)
            gw = dw.view(ldc, 3, 3, cx)[:co, :, :, :weight.shape[1]].permute(0, 3, 1, 2).contiguous()
            if ctx.needs_input_grad[2]:
                gb = cs[:co].contiguous()
        elif ctx.needs_input_grad[2]:
            gb = ops.colsum(g)[:co].contiguous()
        return gx, gw, gb, None, None, None, None


# The training linears' forward and input-gradient GEMMs as SPLIT3 products on the bf16 MFMA (round 6):
# fp32-accurate (ops.linear_split3; against fp64 at or below the fp32-MFMA GEMM's error without a
# residual, <= 1.75x with one, tests/test_gpu_kernels.py) where the 256 x 256 tiles fill the chip
# (engine._split3_fills); the operand is split by one mhada_split3_rows pass, the weights once per
# parameter version.  False: the fp32-MFMA GEMMs.
TRAIN_SPLIT3 = True


def _split3_w(weight: torch.Tensor, transposed: bool) -> torch.Tensor:
    """ops.split3_weight of W (forward, [N][6 K0]) or of W^T (input gradient, [K0][6 N]), cached per
    weight tensor (_pack_slot) and rebuilt when its version changes (every optimizer step)."""
    cache = _pack_slot(weight)
    key = ("s3t",) if transposed else ("s3",)
    hit = cache.get(key)
    if hit is not None and hit[0] == weight._version:
        return hit[1]
    w6 = ops.split3_weight_dev(weight.detach().contiguous(), transposed)
    cache[key] = (weight._version, w6)
    return w6


def _split3_ok(M: int, N: int, K0: int, dev: torch.device) -> bool:
    from .engine import _split3_fills
    return TRAIN_SPLIT3 and N > 128 and K0 % 64 == 0 and _split3_fills(M, N, dev)


# A tensor that the producing SPLIT3 GEMM also wrote as its three bf16 planes (ops.linear_split3(both=True))
# carries them here, with the tensor's _version at the time: the consuming LinearFn then skips its
# mhada_split3_rows pass.  Forward: MLP1's ReLU output for MLP2; backward: MLP2's input gradient (MLP1's
# output gradient, the ReLU mask applied) for MLP1's input-gradient GEMM.  Missing or stale: split again.
PLANES_HANDOFF_ON = True  # False: every SPLIT3 LinearFn splits its operand itself (A/B)
_PLANES_ATTR = "_mhada_split3_planes"
PLANES_HANDOFF = {"used": 0, "split": 0}


def _attach_planes(t: torch.Tensor, planes: torch.Tensor) -> None:
    setattr(t, _PLANES_ATTR, (planes, t._version))


def _planes_of(t: torch.Tensor) -> torch.Tensor:
    hit = getattr(t, _PLANES_ATTR, None)
    if hit is not None:
        delattr(t, _PLANES_ATTR)  # one consumer; do not keep the planes alive with a saved tensor
        if hit[1] == t._version and hit[0].shape == (3, *t.shape):
            PLANES_HANDOFF["used"] += 1
            return hit[0]
    PLANES_HANDOFF["split"] += 1
    return ops.split3_rows(t)


class LinearFn(torch.autograd.Function):
    """y = act(x W^T + b) (+ residual) on contiguous fp32 rows x [M][K], W [N][K] (nn.Linear
    layout).  ``residual`` [M][N] (no ReLU with it): the add of a residual stream fused into the
    GEMM epilogue (the reference's ``t + f(t)``); its gradient is gy itself.  Forward and input
    gradient run as SPLIT3 GEMMs where TRAIN_SPLIT3 and the shape allow (_split3_ok)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu: bool, grad_masked: bool = False, relu_input: bool = False,
                residual=None, planes_out: bool = False):
        x = x.contiguous()
        if residual is not None and relu:
            raise ValueError("LinearFn: a fused residual follows a ReLU-free linear")
        M, K0 = x.shape
        N = weight.shape[0]
        res = None if residual is None else residual.detach().contiguous()
        # planes_out: y's consumer is a SPLIT3 LinearFn — write y's planes from this epilogue as well
        ctx.s3_in = x.dtype == torch.float32 and _split3_ok(M, N, K0, x.device)
        if ctx.s3_in:
            y = ops.linear_split3(_planes_of(x), _split3_w(weight, False), bias.detach().contiguous(), F32,
                                  residual=res, relu=relu, both=planes_out and PLANES_HANDOFF_ON)
            if planes_out and PLANES_HANDOFF_ON:
                y, yp = y
                _attach_planes(y, yp)
        else:
            y = ops.linear(x, weight.detach().contiguous(), bias.detach().contiguous(), F32, relu=relu, residual=res)
        ctx.save_for_backward(x, weight, y if (relu and not grad_masked) else None)
        # grad_masked: y's only consumer is a LinearFn(relu_input=True), whose input-gradient GEMM
        # applies this ReLU's adjoint in its epilogue (mhada_gemm relu = 2): no relu_bwd pass here
        ctx.relu, ctx.grad_masked, ctx.relu_input = relu, grad_masked, relu_input
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, y = ctx.saved_tensors
        g = gy.contiguous()
        if ctx.relu and not ctx.grad_masked:
            g = ops.relu_bwd(g, y)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            M, N = g.shape
            K0 = weight.shape[1]
            if _split3_ok(M, K0, N, g.device):
                # relu_input with a SPLIT3 forward: x came from a SPLIT3 LinearFn(planes_out) whose
                # input-gradient GEMM is SPLIT3 too (same M, N) — hand it gx's planes
                both = PLANES_HANDOFF_ON and ctx.relu_input and ctx.s3_in and _split3_ok(M, N, K0, g.device)
                gx = ops.linear_split3(_planes_of(g), _split3_w(weight, True), None, F32,
                                       relu_mask=x if ctx.relu_input else None, both=both)
                if both:
                    gx, gp = gx
                    _attach_planes(gx, gp)
            else:
                gx = ops.linear(g, weight.detach().t().contiguous(), None, F32, relu_mask=x if ctx.relu_input else None)
        if ctx.needs_input_grad[1]:
            M, N = g.shape
            gw, cs = ops.gemm_tn(g, x, M=N, N=x.shape[1], K=M, lda=N, ldb=x.shape[1], b_mode=A_ROWS, colsum=True)
            if ctx.needs_input_grad[2]:
                gb = cs
        elif ctx.needs_input_grad[2]:
            gb = ops.colsum(g)
        return gx, gw, gb, None, None, None, gy if ctx.needs_input_grad[6] else None, None


def linear(x2d: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, relu: bool = False,
           grad_masked: bool = False, relu_input: bool = False, residual: torch.Tensor = None,
           planes_out: bool = False) -> torch.Tensor:
    return LinearFn.apply(x2d, weight, bias, relu, grad_masked, relu_input, residual, planes_out)


class InstanceNormTokensFn(torch.autograd.Function):
    """F.instance_norm (no affine, eps 1e-5, biased variance; adaDecoder.py:147-149,188-190) on
    token-major rows x [B][N][C]: mhada_instnorm_stats (fixed-order fp64 partials) +
    mhada_rows_normalize.  Backward: dx = rstd (dy - mean_N(dy) - y mean_N(dy y)).  Working on the
    token-major storage of the block's channels-last features avoids the NCHW <-> NHWC copies of
    aten's instance_norm."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x):
        x = x.contiguous()
        mu, rs = ops.instnorm_stats(x)
        y = ops.rows_normalize(x, mu, rs)
        ctx.save_for_backward(y, rs)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        y, rs = ctx.saved_tensors
        return ops.instnorm_bwd(dy.contiguous(), y, rs)


def instance_norm_tokens(x: torch.Tensor) -> torch.Tensor:
    return InstanceNormTokensFn.apply(x)


class LayerNormFn(torch.autograd.Function):
    """nn.LayerNorm (vit.py:54-55,58,62; the EncoderBlock's ln1 / ln2, eps 1e-6) on token rows
    [M][C] fp32: mhada_layernorm_fwd (row statistics kept) and mhada_layernorm_bwd (dx per row,
    dgamma / dbeta as fixed-order column sums)."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, weight, bias, eps: float, planes_for_n: int = 0):
        x = x.contiguous()
        # planes_for_n: y feeds a LinearFn with that many outputs — write its SPLIT3 planes here when
        # that linear runs SPLIT3 (the plane hand-off)
        M, C = x.shape
        if planes_for_n and PLANES_HANDOFF_ON and _split3_ok(M, planes_for_n, C, x.device):
            y, st, pl = ops.layernorm_fwd(x, weight.detach().contiguous(), bias.detach().contiguous(), eps, planes=True)
            _attach_planes(y, pl)
        else:
            y, st = ops.layernorm_fwd(x, weight.detach().contiguous(), bias.detach().contiguous(), eps)
        ctx.save_for_backward(x, st, weight)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        x, st, weight = ctx.saved_tensors
        dx, dg, db = ops.layernorm_bwd(x, dy.contiguous(), st, weight.detach().contiguous())
        return dx, dg, db, None, None


def layernorm(x2d: torch.Tensor, ln: torch.nn.LayerNorm, planes_for_n: int = 0) -> torch.Tensor:
    return LayerNormFn.apply(x2d, ln.weight, ln.bias, ln.eps, planes_for_n)


class PosEmbedFn(torch.autograd.Function):
    """PosEmbedding (vit.py:81-102): the (1, C, bh, bw) table bilinearly resized
    (align_corners=False) to the token grid, token-major [h*w][C] — mhada_pos_embed forward, the
    deterministic gather adjoint mhada_pos_embed_bwd backward."""

    @staticmethod
    def forward(ctx, pos, h: int, w: int):
        ctx.shape = pos.shape
        ctx.hw = (h, w)
        return ops.pos_embed(pos.detach().float().contiguous(), h, w)

    @staticmethod
    def backward(ctx, g):
        h, w = ctx.hw
        _, C, bh, bw = ctx.shape
        return ops.pos_embed_bwd(g.contiguous().view(h, w, C), bh, bw), None, None


def pos_embed(pos: torch.Tensor, h: int, w: int) -> torch.Tensor:
    return PosEmbedFn.apply(pos, h, w)


class HeadProjFn(torch.autograd.Function):
    """The per-head 1x1 convs of AdaAttnMultiHead (adaDecoder.py:143-145,188-190: f/g/h_list[i] on
    channel slice i) as ONE grouped GEMM over the heads: token rows x [T][H*64], stacked weights
    [H][64][64] and biases [H][64] -> y [H][T][64] (head-major: the (head, batch) order the
    training attention takes).  Backward: dX as the grouped GEMM with the transposed head weights
    (written straight into each head's column block), dW per head on the TN kernel, db a column
    sum.  1/8 of the block-diagonal 512x512 product's FLOPs in each direction."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, weight, bias):
        x = x.contiguous()
        T, C = x.shape
        H = weight.shape[0]
        if C != 64 * H or weight.shape[1:] != (64, 64):
            raise ValueError("HeadProjFn: x [T][64H], weight [H][64][64]")
        y = torch.empty(H, T, 64, device=x.device, dtype=F32)
        ops.gemm(a=x, w=weight.detach().contiguous(), c=y, M=T, N=64, K=64, compute=F32, lda=C, sa=(64, 0),
                 nb=(H, 1), ldw=64, sw=(4096, 0), bias=bias.detach().contiguous(), sb=(64, 0), ldc=64,
                 sc=(T * 64, 0))
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        T, C = x.shape
        H = weight.shape[0]
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty(T, C, device=x.device, dtype=F32)
            ops.gemm(a=gy, w=weight.detach().transpose(1, 2).contiguous(), c=gx, M=T, N=64, K=64, compute=F32,
                     lda=64, sa=(T * 64, 0), nb=(H, 1), ldw=64, sw=(4096, 0), ldc=C, sc=(64, 0))
        if ctx.needs_input_grad[1]:
            # all heads in one batched TN launch (head i: A = gy[i], B = x[:, 64i:]), the bias
            # gradients from the same pass
            gw, cs = ops.gemm_tn(gy, x, M=64, N=64, K=T, lda=64, ldb=C, b_mode=A_ROWS, colsum=True, nb=H,
                                 sza=T * 64, szb=64)
            if ctx.needs_input_grad[2]:
                gb = cs
        elif ctx.needs_input_grad[2]:
            gb = gy.sum(dim=1)
        return gx, gw, gb


def head_proj(x2d: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    return HeadProjFn.apply(x2d, weight, bias)


class BatchAxisAttnFn(torch.autograd.Function):
    """The core of nn.MultiheadAttention(batch_first=False) on a (B, N, C) tensor (vit.py:48,59):
    per token and head, softmax over the L = B images of (q/8) k^T, times v.  qkv [L][N][3C]
    fp32 (the packed in-projection output) -> [L][N][C]; mhada_vit_batch_attn forward,
    mhada_vit_batch_attn_bwd backward."""

    @staticmethod
    def forward(ctx, qkv, heads: int, groups: int = 1, L: int = 0):
        """qkv [L][N][3C], or [L N][3C] rows with L given (the QKV LinearFn's own output tensor: its
        gradient then reaches that LinearFn as the same tensor, carrying the SPLIT3 plane hand-off)."""
        qkv = qkv.contiguous()
        rows2d = qkv.dim() == 2
        q3 = qkv.view(L, qkv.shape[0] // L, qkv.shape[1]) if rows2d else qkv
        Lq, N, _ = q3.shape
        ctx.save_for_backward(q3)
        ctx.heads, ctx.groups, ctx.rows2d = heads, groups, rows2d
        return ops.vit_batch_attn(q3, Lq, N, heads, groups)

    @staticmethod
    def backward(ctx, gout):
        (qkv,) = ctx.saved_tensors
        L, N, C3 = qkv.shape
        # rows: the producing QKV LinearFn's input-gradient GEMM takes dqkv's planes when it is SPLIT3
        if ctx.rows2d and PLANES_HANDOFF_ON and _split3_ok(L * N, C3 // 3, C3, qkv.device):
            dqkv, pl = ops.vit_batch_attn_bwd(qkv, gout.contiguous(), L, N, ctx.heads, ctx.groups, planes=True)
            dq2 = dqkv.view(L * N, C3)
            _attach_planes(dq2, pl)
            return dq2, None, None, None
        dqkv = ops.vit_batch_attn_bwd(qkv, gout.contiguous(), L, N, ctx.heads, ctx.groups)
        return (dqkv.view(L * N, C3) if ctx.rows2d else dqkv), None, None, None


class PatchEmbedFn(torch.autograd.Function):
    """PatchEmbedding conv 8x8 / stride 8 (vit.py:105-117): img (B, 3, H, W) fp32 -> tokens
    [B][N][C]; weight (C, 3, 8, 8).  Gradients for the weight and bias only."""

    @staticmethod
    def forward(ctx, img, weight, bias):
        img = img.float().contiguous()
        C = weight.shape[0]
        y = ops.patch_embed(img, weight.detach().reshape(C, -1).contiguous(), bias.detach().float().contiguous(), None)
        ctx.save_for_backward(img, weight)
        return y

    @staticmethod
    def backward(ctx, gy):
        img, weight = ctx.saved_tensors
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("PatchEmbedFn: no input-image gradient (training inputs are data)")
        B, Ci, H, W = img.shape
        C = weight.shape[0]
        g = gy.contiguous().view(-1, C)
        gw = gb = None
        if ctx.needs_input_grad[1]:
            gw, cs = ops.gemm_tn(g, img, M=C, N=64 * Ci, K=g.shape[0], lda=C, b_mode=A_PATCH8, img=(Ci, H, W),
                                 colsum=True)
            gw = gw.view_as(weight)
            if ctx.needs_input_grad[2]:
                gb = cs
        elif ctx.needs_input_grad[2]:
            gb = ops.colsum(g)
        return None, gw, gb


class MaxPool2Fn(torch.autograd.Function):
    """MaxPool2d(2, 2) on NHWC.  relu_input: x is a ReLU output consumed only by this pool, so the
    backward also applies the ReLU adjoint and the producing Conv3x3Fn (grad_masked=True) skips it."""

    @staticmethod
    def forward(ctx, x, relu_input: bool = False):
        ctx.save_for_backward(x)
        ctx.relu_input = relu_input
        return ops.maxpool2(x)

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        return ops.maxpool2_bwd(x, gy.contiguous(), ctx.relu_input), None


class Upsample2xFn(torch.autograd.Function):
    """Bilinear x2 on NHWC.  relu_input: x is the ReLU output of a Conv3x3Fn(grad_masked=True)
    consumed only here, and the backward applies that ReLU's adjoint too."""

    @staticmethod
    def forward(ctx, x, relu_input: bool = False):
        ctx.relu_input = relu_input
        if relu_input:
            ctx.save_for_backward(x)
        return ops.upsample2x(x)

    @staticmethod
    def backward(ctx, gy):
        relu_x = ctx.saved_tensors[0] if ctx.relu_input else None
        return ops.upsample2x_bwd(gy.contiguous(), relu_x), None


class VggInputFn(torch.autograd.Function):
    """imageNet1k_normalize (vgg19.py:6-12) + NCHW -> NHWC with channels padded to 32."""

    @staticmethod
    def forward(ctx, img):
        return ops.vgg_input(img.float().contiguous(), 32)

    @staticmethod
    def backward(ctx, g):
        return ops.vgg_input_bwd(g.contiguous())


class FeatureLossFn(torch.autograd.Function):
    """The loss terms of train_image.py on ONE VGG feature map x (an NCHW view of NHWC storage):
      l_mean = mse(mean_hw(x), ref_mean), l_std = mse(std_hw(x), ref_std)  (lossfn.py:7-23; ref given)
      l_mse  = mse(x, t)                            (lossfn.py:26-34 and 41-47; t given)
    On the device the forward takes the three reductions from ONE pass (mhada_feat_stats: fp64
    partial sums, fixed order — the aten values up to their fp32 summation order); on the CPU the
    reference's own aten expressions.  The backward writes dL/dx = g_mean 2(mu - mu_r) / (BC HW) + g_std 2(sd - sd_r)(x - mu) / (BC (HW-1) sd)
    + g_mse 2(x - t) / numel in ONE mhada_feat_loss_bwd pass, in place of ATen's mse / std / mean
    backward chains and the adds that sum the terms of a feature map."""

    @staticmethod
    def forward(ctx, x, ref_mean, ref_std, t, relu_input: bool = False):
        if any(ctx.needs_input_grad[1:4]):
            raise ValueError("FeatureLossFn: the reference statistics and the target take no gradient")
        # relu_input: x is a ReLU output whose producer (a Conv3x3Fn(grad_masked=True), see
        # vgg19_forward(masked_features=True)) leaves the ReLU adjoint to its consumers
        ctx.relu_input = relu_input
        ctx.set_materialize_grads(False)
        zero = x.new_zeros(())
        lm = ls = lmse = zero
        mu = sd = None
        xs, ts = _nhwc(x), None if t is None else _nhwc(t)
        if xs is not None and (t is None or ts is not None) and (ref_mean is not None or t is not None):
            mu, sd, m = ops.feat_stats(xs, ts, stats=ref_mean is not None)
            if ref_mean is not None:
                lm = F.mse_loss(mu, ref_mean)
                ls = F.mse_loss(sd, ref_std)
            if t is not None:
                lmse = m
        else:
            if ref_mean is not None:
                mu = x.mean(dim=(2, 3))
                sd = x.std(dim=(2, 3))
                lm = F.mse_loss(mu, ref_mean)
                ls = F.mse_loss(sd, ref_std)
            if t is not None:
                lmse = F.mse_loss(x, t)
        ctx.save_for_backward(x, t, mu, sd, ref_mean, ref_std)
        return lm, ls, lmse

    @staticmethod
    def backward(ctx, g_mean, g_std, g_mse):
        x, t, mu, sd, rm, rs = ctx.saved_tensors
        B, C, H, W = x.shape
        P = H * W
        xs = x.permute(0, 2, 3, 1)
        xs = xs if xs.is_contiguous() else xs.contiguous()
        alpha = beta = None
        if mu is not None and (g_mean is not None or g_std is not None):
            zero = x.new_zeros(())
            gm = g_mean if g_mean is not None else zero
            gs = g_std if g_std is not None else zero
            alpha = (gm * (2.0 / (B * C * P)) * (mu - rm)).contiguous()
            beta = (gs * (2.0 / (B * C * (P - 1))) * (sd - rs) / sd).contiguous()
        tt = None
        if t is not None and g_mse is not None:
            tt = t.permute(0, 2, 3, 1)
            tt = tt if tt.is_contiguous() else tt.contiguous()
        if alpha is None and tt is None:
            if ctx.relu_input:
                raise RuntimeError("FeatureLossFn(relu_input=True) must return the masked gradient")
            return None, None, None, None, None
        kp = g_mse.reshape(1).float().contiguous() if tt is not None else None
        g = ops.feat_loss_bwd(xs, mu.contiguous() if alpha is not None else None, alpha, beta, tt, 2.0 / x.numel(), kp,
                              relu=ctx.relu_input)
        return g.permute(0, 3, 1, 2), None, None, None, None


def _nhwc(x: torch.Tensor):
    """x's NHWC storage as a contiguous [B][H][W][C] fp32 device view, or None (CPU, other layout)."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] % 4:
        return None
    v = x.permute(0, 2, 3, 1)
    return v if v.is_contiguous() else None


def feature_mean_std(x: torch.Tensor):
    """(x.mean(dim=(2, 3)), x.std(dim=(2, 3))) of a feature map: one mhada_feat_stats pass on the
    device (calc_mean_std of lossfn.py:10-19 for the style targets)."""
    xs = _nhwc(x)
    if xs is None:
        return x.mean(dim=(2, 3)), x.std(dim=(2, 3))
    mu, sd, _ = ops.feat_stats(xs)
    return mu, sd


def feature_loss_terms(x, ref_mean=None, ref_std=None, t=None, relu_input: bool = False):
    """(l_mean, l_std, l_mse) of one feature map (FeatureLossFn)."""
    return FeatureLossFn.apply(x, ref_mean, ref_std, t, relu_input)


def _cached_build(weight: torch.Tensor, key: tuple, build) -> torch.Tensor:
    """A derived layout of a frozen weight, cached like _cached; built per call when trainable."""
    if weight.requires_grad:
        return build()
    cache = _pack_slot(weight)
    hit = cache.get(key)
    if hit is not None and hit[0] == weight._version:
        return hit[1]
    w = build()
    cache[key] = (weight._version, w)
    return w


class Out3Fn(torch.autograd.Function):
    """The decoder's last layer (conv.py:94, ConvReLU(64, 3): ReflectionPad2d(1) -> Conv2d(64, 3, 3)
    -> ReLU) from NHWC x [B][H][W][64] straight to the NCHW image [B][3][H][W]: forward on
    mhada_conv3x3_out3 (the inference kernel), backward on mhada_out3_dgrad (ReLU, transposed conv
    and reflection-pad adjoints in one pass) and mhada_out3_wgrad."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu_input: bool = False):
        # relu_input: x is the ReLU output of a Conv3x3Fn(grad_masked=True) whose only consumer is
        # this layer, and the input gradient carries that ReLU's adjoint too
        wf = weight.detach().permute(2, 3, 1, 0).float().contiguous()  # [tap][ci][co]
        y = ops.conv3x3_out3(x, wf, bias.detach().float().contiguous())
        ctx.save_for_backward(x, weight, y)
        ctx.relu_input = relu_input
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, y = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            wd = weight.detach().permute(2, 3, 0, 1).reshape(9, 3, 64).float().contiguous()  # [tap][co][ci]
            gx = ops.out3_dgrad(gy, y, wd, x if ctx.relu_input else None)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dw, db = ops.out3_wgrad(x, gy, y, bias=ctx.needs_input_grad[2])
            gw = dw if ctx.needs_input_grad[1] else None
            gb = db
        return gx, gw, gb, None


def _out3_eligible(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    return (x.is_cuda and x.dtype == F32 and x.dim() == 4 and x.shape[-1] == 64 and x.shape[1] >= 2
            and x.shape[2] >= 2 and x.is_contiguous() and tuple(conv.weight.shape) == (3, 64, 3, 3)
            and conv.bias is not None)


class VggStemFn(torch.autograd.Function):
    """VGG19's input normalisation and first layer (vgg19.py:10-11,25-26: imageNet1k_normalize ->
    Conv2d(3, 64, 3, padding=1) -> ReLU) with frozen weights: the forward is VggInputFn + the
    zero-padded conv; the backward is ONE mhada_vgg_stem_dgrad pass (ReLU adjoint, the 64 -> 3
    transposed conv, the normalisation adjoint) in place of relu_bwd, a 64 -> 32-channel GEMM conv
    and vgg_input_bwd."""

    @staticmethod
    def forward(ctx, img, weight, bias):
        x = ops.vgg_input(img.float().contiguous(), 32)
        B, H, W, cx = x.shape
        y = torch.empty(B, H, W, 64, device=x.device, dtype=F32)
        wf = _cached(weight, "f", cx)
        ops.conv3x3(x, wf, bias.detach().float().contiguous(), F32, upsample=False, relu=True, pad_mode="zero",
                    pad=1, out=y, wino_u=_wino(weight, "f", wf, cx))
        ctx.save_for_backward(weight, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        weight, y = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None
        wd = _cached_build(weight, ("stem_d",), lambda: weight.detach()[:, :3].flip(2, 3).permute(2, 3, 0, 1)
                           .reshape(9, 64, 3).float().contiguous())
        return ops.vgg_stem_dgrad(gy.contiguous(), y, wd), None, None


def _stem_eligible(img: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    return (img.is_cuda and img.dim() == 4 and img.shape[1] == 3 and tuple(conv.weight.shape) == (64, 3, 3, 3)
            and conv.bias is not None and not conv.weight.requires_grad and not conv.bias.requires_grad)


def conv3x3(x, conv: torch.nn.Conv2d, pad_mode: str, relu: bool = True, grad_masked: bool = False,
            relu_input: bool = False):
    return Conv3x3Fn.apply(x, conv.weight, conv.bias, pad_mode, relu, grad_masked, relu_input)


def nchw_to_nhwc(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 2, 3, 1).contiguous()


def nhwc_to_nchw(x: torch.Tensor) -> torch.Tensor:
    """An NCHW view of NHWC storage (channels_last strides; no copy)."""
    return x.permute(0, 3, 1, 2)


def decoder_forward(dec, x_nchw: torch.Tensor, order) -> torch.Tensor:
    """Decoder.forward (conv.py:96-100) on the HIP training kernels; ``order`` lists
    (sequence name, index, upsample-after) as autograd_path.DECODER_ORDER."""
    x = nchw_to_nhwc(x_nchw.float())
    last = getattr(dec, order[-1][0])[order[-1][1]].conv.conv
    masked = False
    relu_in = False  # x is the ReLU output of the previous conv, consumed only by this conv
    for i, (seq, idx, up) in enumerate(order):
        conv = getattr(dec, seq)[idx].conv.conv
        if i == len(order) - 1 and not up and (masked or _out3_eligible(x, conv)):
            return Out3Fn.apply(x, conv.weight, conv.bias, masked)  # conv3.1: 64 -> 3, NCHW out
        if i == len(order) - 1 and masked:
            raise RuntimeError("decoder_forward: the masked layer's consumer must be Out3Fn")
        # the layer feeding conv3.1 directly (conv3.0) leaves its ReLU adjoint to Out3Fn's dgrad;
        # its output (NHWC, 64 channels, same H x W) then meets every _out3_eligible condition
        masked = (i == len(order) - 2 and not up and not order[-1][2] and conv.weight.shape[0] == 64
                  and x.is_cuda and x.dtype == F32 and x.shape[1] >= 2 and x.shape[2] >= 2
                  and tuple(last.weight.shape) == (3, 64, 3, 3) and last.bias is not None)
        # a layer followed by the bilinear x2 leaves its ReLU adjoint to the upsample's backward, one
        # followed by another conv3x3 of this loop to that conv's input gradient (relu_input)
        nxt_conv = (not up and not masked and x.is_cuda and i + 1 < len(order) - 1)
        x = conv3x3(x, conv, "reflect", relu=True, grad_masked=masked or (up and x.is_cuda) or nxt_conv,
                    relu_input=relu_in)
        relu_in = nxt_conv
        if up:
            x = Upsample2xFn.apply(x, x.is_cuda)
    return x.permute(0, 3, 1, 2).contiguous()


def vgg19_forward(vgg, img: torch.Tensor, convs, pools, slices, masked_features: bool = False) -> Dict[str, torch.Tensor]:
    """VGG19.forward (vgg19.py:42-70) on the HIP kernels: relu1_1 .. relu5_1 as NCHW views of
    NHWC storage.  masked_features (the Trainer's fused losses only): the caller guarantees that every
    gradient reaching a feature map relu2_1 .. relu5_1 comes from a FeatureLossFn(relu_input=True),
    so the convs producing them skip their ReLU adjoint: the loss backward applies it, and the next
    slice's first conv applies it in its dgrad (relu_input)."""
    x = None
    relu_to_pool = False
    relu_in = False
    feats = {}
    for s, (a, b) in enumerate(slices, start=1):
        seq = getattr(vgg, f"slice{s}")
        for i in range(a, b):
            if i in convs:
                conv = getattr(seq, str(i))
                if x is None:
                    if _stem_eligible(img, conv):
                        x = VggStemFn.apply(img, conv.weight, conv.bias)
                        continue
                    x = VggInputFn.apply(img)
                # a conv whose ReLU output feeds only the next pool (vgg19 cfg E: conv1_2, conv2_2,
                # conv3_4, conv4_4) leaves its ReLU adjoint to the pool's backward
                pooled = (i + 2) in pools and i + 2 < b
                # a conv whose ReLU output feeds only the next conv of the same slice (conv3_2, 3_3,
                # 4_2, 4_3: not a slice end, so not a loss feature) leaves it to that conv's dgrad
                chained = (i + 2) in convs and i + 2 < b and x.is_cuda
                feature = masked_features and s >= 2 and i + 2 == b and x.is_cuda  # relu2_1 .. relu5_1
                x = conv3x3(x, conv, "zero", relu=True, grad_masked=pooled or chained or feature, relu_input=relu_in)
                relu_in = chained or feature
                relu_to_pool = pooled
            elif i in pools:
                x = MaxPool2Fn.apply(x, relu_to_pool)
                relu_to_pool = False
            # ReLU modules are fused into the conv epilogue
        feats[f"relu{s}_1"] = nhwc_to_nchw(x)
    return feats
