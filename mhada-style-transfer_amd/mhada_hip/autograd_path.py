"""Differentiable forward passes for the training path.

When a forward needs gradients (``torch.is_grad_enabled()`` and a parameter or input requires
grad — ``train_image.py:93-144``, feature-inversion scripts) or runs on CPU tensors (the
reference scripts' no-GPU branch, ``infer_image.py:48``), the ``network`` modules route here
instead of to the inference engine.  On ROCm device tensors every conv / linear / attention /
normalisation runs on the HIP training kernels through the autograd Functions of
``train_fns`` (and ``MHAdaAttnFn``: csrc/attn_train.hip forward + backward); on CPU tensors the
same functions evaluate the reference's aten expression.
Each function evaluates the reference algorithm on the module's own parameter containers
(the same ``nn.Conv2d`` / ``nn.MultiheadAttention`` / ``nn.Linear`` / ``nn.LayerNorm`` objects
whose state_dict keys match the reference), so autograd reaches exactly those parameters.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F

from . import ops

# "hip": the MHAda attention core trains on the HIP kernels; "torch": plain autograd (A/B, tests)
TRAIN_ATTN = "hip"

# decoder layers and whether bilinear x2 follows them (conv.py:78-94)
DECODER_ORDER = (("conv1", 0, True), ("conv1", 1, False), ("conv1", 2, False), ("conv1", 3, False),
                 ("conv1", 4, True), ("conv2", 0, False), ("conv2", 1, True), ("conv3", 0, False),
                 ("conv3", 1, False))


def needs_grad(module: torch.nn.Module, *xs) -> bool:
    if not torch.is_grad_enabled():
        return False
    if any(isinstance(x, torch.Tensor) and x.requires_grad for x in xs):
        return True
    return any(p.requires_grad for p in module.parameters())


def _vit_forward_hip(vit, x: torch.Tensor, groups: int = 1) -> List[torch.Tensor]:
    """VisionTransformer.forward on the HIP training kernels (train_fns): patch embedding and
    every Linear (MHA in/out projections, MLP with fused ReLU) on mhada_gemm forward and
    mhada_gemm / mhada_gemm_tn / mhada_colsum backward; LayerNorm on mhada_layernorm_fwd/_bwd; the
    pos-embed resize on mhada_pos_embed and its gather adjoint; the batch-axis attention core
    (L = B <= 8 keys per token) on mhada_vit_batch_attn(_bwd).  ``groups`` > 1: x holds that many
    calls' batches back to back, attended separately (vit_forward)."""
    from . import train_fns
    B, _, H, W = x.shape
    p = vit.patch_size
    h, w = H // p, W // p
    N = h * w
    t = train_fns.PatchEmbedFn.apply(x, vit.patch_embedding.conv_proj.weight, vit.patch_embedding.conv_proj.bias)
    C = t.shape[2]
    if vit.pos_embedding is not None:
        t = t + train_fns.pos_embed(vit.pos_embedding.pos_embed, h, w).view(1, N, C)
    outs = []
    ln_hip = C in (256, 512, 1024)
    for blk in vit.encoder:
        att = blk.attention
        heads = att.num_heads
        d = C // heads
        y = train_fns.layernorm(t.reshape(B * N, C), blk.ln1, 3 * C) if ln_hip else blk.ln1(t).reshape(B * N, C)
        qkv = train_fns.linear(y, att.in_proj_weight, att.in_proj_bias)
        if d == 64 and B // groups <= 8:  # the batch-axis attention core on HIP (L = B keys per token)
            o = train_fns.BatchAxisAttnFn.apply(qkv, heads, groups, B).reshape(B * N, C)
        else:
            Lg = B // groups
            q, k, v = (z.reshape(groups, Lg, N, heads, d).permute(0, 2, 3, 1, 4)  # (G, N, H, L, d)
                       for z in qkv.split(C, dim=1))
            a = torch.softmax(torch.matmul(q, k.transpose(-1, -2)) * (d ** -0.5), dim=-1)
            o = torch.matmul(a, v).permute(0, 3, 1, 2, 4).reshape(B * N, C)
        # the residual adds of vit.py:60-61 fused into the out-projection / MLP2 GEMM epilogues
        t = train_fns.linear(o, att.out_proj.weight, att.out_proj.bias, residual=t.reshape(B * N, C)).view(B, N, C)
        y2 = train_fns.layernorm(t.reshape(B * N, C), blk.ln2, 4 * C) if ln_hip else blk.ln2(t).reshape(B * N, C)
        # MLP1's ReLU adjoint is applied by MLP2's input-gradient GEMM (its only consumer)
        m = train_fns.linear(y2, blk.mlp[0].weight, blk.mlp[0].bias, relu=True, grad_masked=True, planes_out=True)
        t = train_fns.linear(m, blk.mlp[2].weight, blk.mlp[2].bias, relu_input=True,
                             residual=t.reshape(B * N, C)).view(B, N, C)
        outs.append(t.permute(0, 2, 1).reshape(B, C, h, w))
    return outs


def vit_forward(vit, x: torch.Tensor, groups: int = 1) -> List[torch.Tensor]:
    """VisionTransformer.forward (vit.py:148-169); the MHA keeps batch_first=False on a
    (B, N, C) tensor, i.e. attends over the batch axis exactly as the reference.  On a ROCm
    device the HIP training kernels run it (_vit_forward_hip); the CPU uses aten.

    ``groups`` > 1: x is that many calls' batches concatenated (B = groups x L); the batch-axis
    attention runs over each call's L images separately, everything else is per token, so the
    outputs are those of the separate calls (Trainer.batch_vit)."""
    if x.is_cuda and vit.patch_size == 8 and not x.requires_grad and \
            isinstance(vit.encoder[0].mlp[1], torch.nn.ReLU) and vit.encoder[0].attention.in_proj_weight is not None:
        return _vit_forward_hip(vit, x, groups)
    if groups > 1:
        parts = [vit_forward(vit, xg) for xg in x.chunk(groups)]
        return [torch.cat(o) for o in zip(*parts)]
    B, _, H, W = x.shape
    p = vit.patch_size
    h, w = H // p, W // p
    t = vit.patch_embedding.conv_proj(x)
    C = t.shape[1]
    t = t.reshape(B, C, h * w).permute(0, 2, 1)
    if vit.pos_embedding is not None:
        pe = vit.pos_embedding.pos_embed
        if (h, w) != tuple(pe.shape[2:]):
            pe = F.interpolate(pe, size=(h, w), mode="bilinear", align_corners=False)
        t = t + pe.expand(B, -1, -1, -1).reshape(B, C, h * w).permute(0, 2, 1)
    outs = []
    for blk in vit.encoder:
        y = blk.ln1(t)
        y, _ = blk.attention(y, y, y, need_weights=False)
        t = y + t
        t = t + blk.mlp(blk.ln2(t))
        outs.append(t.permute(0, 2, 1).reshape(B, C, h, w))
    return outs


def _softmax_or_cosine(q, k, activation: str):
    if activation == "softmax":
        return torch.softmax(torch.bmm(q, k), dim=-1)  # adaDecoder.py:16-17, no 1/sqrt(d)
    s = torch.bmm(q, k) / torch.bmm(q.norm(dim=-1, keepdim=True), k.norm(dim=1, keepdim=True)) + 1
    return s / s.sum(dim=-1, keepdim=True)  # adaDecoder.py:24-34


class MHAdaAttnFn(torch.autograd.Function):
    """The attention core of adaDecoder.py:186-198 on the HIP training kernels
    (csrc/attn_train.hip): out' = sqrt(max(E2' - M'^2, 1e-6)) * x + M' with M' = A V',
    E2' = A V'^2, A = softmax(q k^T).  q, x (BH, Nc, 64); k, v (BH, Ns, 64), v centred.
    A is never stored: the backward recomputes it from the saved row normaliser."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, q, k, v, x):
        q, k, v, x = (t.contiguous() for t in (q, k, v, x))
        out, mo, lse = ops.attn_train_fwd(q, k, v, x)
        ctx.save_for_backward(q, k, v, x, mo, lse)
        return out

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dout):
        q, k, v, x, mo, lse = ctx.saved_tensors
        # S = sqrt(max(E2' - M'^2, 1e-6)), out' = S x + M': dx = dout S, dVar = dout x / (2 S) where
        # the clamp is inactive, dM' = dout - 2 M' dVar, dd = rowsum(dM' M' + dVar E2')  (one kernel)
        dx, dmo, dd = ops.attn_train_bwd_prep(dout.contiguous(), x, mo)
        dq, dk, dv = ops.attn_train_bwd(q, k, v, lse, dmo, dd)
        return dq, dk, dv, dx


def _fused_train_attn(blk, fc) -> bool:
    """The HIP training kernels compute in fp32.  An fp32 input takes this path; so does any
    floating input inside a CUDA autocast region (MHAdaAttnFn's custom_fwd casts its operands to
    fp32 there).  Outside autocast a bf16 / fp16 / fp64 block input (model.half(), a gradcheck)
    runs the aten formula: the token-path statistics kernels read fp32 only."""
    return (fc.is_cuda and (fc.dtype == torch.float32 or (fc.is_floating_point() and torch.is_autocast_enabled("cuda")))
            and blk.activation_name == "softmax" and blk.head_dim == 64 and TRAIN_ATTN != "torch")


def _head_proj(mods, t: torch.Tensor, H: int) -> torch.Tensor:
    """Per-head 1x1 convs (adaDecoder.py:188-190, f/g/h_list[i] on channel slice i) on the
    modules' own parameters.  On a ROCm device: ONE grouped GEMM over the heads on the HIP
    kernels (train_fns.head_proj; the gradients reach each head's weight through torch.stack),
    (B, 64H, h, w) -> (H*B, h*w, 64) in HEAD-major order.  On the CPU: a head-batched matmul,
    (B*H, h*w, 64) batch-major.  The attention core treats (head, batch) pairs independently;
    _heads_rows and the out_conv gather follow the same order."""
    B, C, h, w = t.shape
    d = C // H
    if t.is_cuda:
        from . import train_fns
        wst = torch.stack([m.weight.reshape(d, d) for m in mods])
        bst = torch.stack([m.bias for m in mods])
        rows = t.permute(0, 2, 3, 1).reshape(B * h * w, C)
        return train_fns.head_proj(rows, wst, bst).view(H * B, h * w, d)
    wgt = torch.stack([m.weight.reshape(d, d) for m in mods], 0)  # (H, out, in)
    bias = torch.stack([m.bias for m in mods], 0).unsqueeze(1)     # (H, 1, out)
    y = torch.matmul(t.reshape(B, H, d, h * w).transpose(2, 3), wgt.transpose(1, 2)) + bias
    return y.reshape(B * H, h * w, d)


def _heads_rows(t: torch.Tensor, H: int, head_major: bool = False) -> torch.Tensor:
    """(B, 64H, h, w) -> (B*H, h*w, 64) contiguous, batch-major or (head_major) (H*B, ...)."""
    B, C, h, w = t.shape
    if head_major:
        return t.reshape(B, H, C // H, h * w).permute(1, 0, 3, 2).reshape(H * B, h * w, C // H).contiguous()
    return t.reshape(B, H, C // H, h * w).transpose(2, 3).reshape(B * H, h * w, C // H).contiguous()


def block_forward_fused(blk, fc: torch.Tensor, fs: torch.Tensor, fcs: torch.Tensor) -> torch.Tensor:
    """AdaAttnMultiHead.forward (adaDecoder.py:162-206) with the per-head 1x1 convs grouped over
    heads (on a ROCm device one grouped GEMM each, head-major operands) and the attention on
    MHAdaAttnFn."""
    B, C, h, w = fc.shape
    H = blk.num_heads
    if fc.is_cuda:  # token-major throughout: the features are channels-last NCHW views
        from . import train_fns
        d = C // H
        tok = lambda t: t.permute(0, 2, 3, 1).reshape(t.shape[0], -1, C)  # noqa: E731
        fct, fst, fcst = tok(fc), tok(fs), tok(fcs)
        ns = fst.shape[1]

        def proj(mods, rows):
            wst = torch.stack([m.weight.reshape(d, d) for m in mods])
            bst = torch.stack([m.bias for m in mods])
            return train_fns.head_proj(rows, wst, bst)  # [H][rows][d]

        q = proj(blk.f_list, train_fns.instance_norm_tokens(fct).view(B * h * w, C)).view(H * B, h * w, d)
        k = proj(blk.g_list, train_fns.instance_norm_tokens(fst).view(B * ns, C)).view(H * B, ns, d)
        v = proj(blk.h_list, fst.reshape(B * ns, C)).view(H * B, ns, d)
        x = train_fns.instance_norm_tokens(fcst).view(B, h * w, H, d).permute(2, 0, 1, 3).reshape(H * B, h * w, d)
    else:
        q = _head_proj(blk.f_list, F.instance_norm(fc), H).contiguous()
        k = _head_proj(blk.g_list, F.instance_norm(fs), H).contiguous()
        v = _head_proj(blk.h_list, fs, H)
        x = _heads_rows(F.instance_norm(fcs), H)
    # V is centred per (head, image, channel) before the moments (E2' - M'^2 without cancellation)
    # and the mean added back: out = S x + A (v - c) + c = S x + A v for ANY per-row-constant c
    # (softmax rows sum to 1; the variance is shift-invariant), so d out / d c = 0 and c is
    # detached — its gradient terms (sum over Nc of dout, minus the mean of dv) are exact zeros the
    # backward would otherwise spend five kernels per block on
    vmu = v.detach().mean(dim=1, keepdim=True)
    o = MHAdaAttnFn.apply(q, k, (v - vmu).contiguous(), x) + vmu
    if fc.is_cuda:  # out_conv (1x1) as a token GEMM on the HIP kernels
        from . import train_fns
        rows = o.view(H, B * h * w, C // H).permute(1, 0, 2).reshape(B * h * w, C)
        y = train_fns.linear(rows, blk.out_conv.weight.view(C, C), blk.out_conv.bias)
        return y.view(B, h, w, C).permute(0, 3, 1, 2)
    o = o.reshape(B, H, h * w, C // H).transpose(2, 3).reshape(B, C, h, w)
    return blk.out_conv(o)


def _cosine_moments(q, k, v):
    """(A V, A V^2) for the cosine activation (adaDecoder.py:20-34) WITHOUT forming A: with unit
    rows q^ and columns k^, A[i][j] = (q^_i . k^_j + 1) / l_i and l_i = q^_i . sum_j k^_j + Ns, so
      A V   = (q^ (K^ V)   + 1 sum_j v_j)   / l,   A V^2 = (q^ (K^ V^2) + 1 sum_j v_j^2) / l
    with d x d products (O(N d^2) instead of the N_c x N_s matrix) — the same quantities as the
    reference expression up to fp32 summation order, and a backward that autograd derives without
    the N_c x N_s intermediates.  q (B, Nc, d), k (B, d, Ns), v (B, Ns, d)."""
    qn = q / q.norm(dim=-1, keepdim=True)
    kn = k / k.norm(dim=1, keepdim=True)
    v2 = v * v
    l = torch.matmul(qn, kn.sum(dim=-1, keepdim=True)) + k.shape[-1]          # (B, Nc, 1)
    m = (torch.bmm(qn, torch.bmm(kn, v)) + v.sum(dim=1, keepdim=True)) / l
    e2 = (torch.bmm(qn, torch.bmm(kn, v2)) + v2.sum(dim=1, keepdim=True)) / l
    return m, e2


def block_forward(blk, fc: torch.Tensor, fs: torch.Tensor, fcs: torch.Tensor) -> torch.Tensor:
    """AdaAttnMultiHead.forward (adaDecoder.py:162-206).  On a ROCm device the cosine activation
    trains on its linear form (_cosine_moments); CPU tensors evaluate the reference expression."""
    if _fused_train_attn(blk, fc):
        return block_forward_fused(blk, fc, fs, fcs)
    B, _, h, w = fc.shape
    d = blk.head_dim
    linear_cos = fc.is_cuda and blk.activation_name == "cosine"
    outs = []
    for i in range(blk.num_heads):
        sl = slice(i * d, (i + 1) * d)
        q = blk.f_list[i](F.instance_norm(fc[:, sl])).reshape(B, d, h * w).permute(0, 2, 1)
        k = blk.g_list[i](F.instance_norm(fs[:, sl]))
        k = k.reshape(B, d, -1)
        v = blk.h_list[i](fs[:, sl]).reshape(B, d, -1).permute(0, 2, 1)
        if linear_cos:
            m, e2 = _cosine_moments(q, k, v)
            s = torch.sqrt((e2 - m * m).clamp(min=1e-6))
        else:
            a = _softmax_or_cosine(q, k, blk.activation_name)
            m = torch.bmm(a, v)
            s = torch.sqrt((torch.bmm(a, v * v) - m * m).clamp(min=1e-6))
        m = m.reshape(B, h, w, d).permute(0, 3, 1, 2)
        s = s.reshape(B, h, w, d).permute(0, 3, 1, 2)
        outs.append(s * F.instance_norm(fcs[:, sl]) + m)
    return blk.out_conv(torch.cat(outs, dim=1))


def decoder_forward(dec, x: torch.Tensor) -> torch.Tensor:
    """Decoder.forward (conv.py:96-100): on a ROCm device the HIP training kernels
    (train_fns: implicit-GEMM conv fwd / dgrad / wgrad, upsample and its adjoint); the CPU
    (test plumbing) evaluates the same expression with aten ops."""
    if x.is_cuda:
        from . import train_fns
        return train_fns.decoder_forward(dec, x, DECODER_ORDER)
    for seq, idx, up in DECODER_ORDER:
        conv = getattr(dec, seq)[idx].conv.conv
        x = F.relu(conv(F.pad(x, (1, 1, 1, 1), mode="reflect")))
        if up:
            x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    return x


def adaformer_forward(ada, fc: Sequence[torch.Tensor], fs: Sequence[torch.Tensor]):
    """AdaAttnTransformerMultiHead.forward (adaDecoder.py:253-268)."""
    fcs = fc[0]
    for i in range(ada.num_layers):
        fcs = block_forward(ada.adaAttnHead[2 * i], fc[i], fs[i], fcs)
        fcs = block_forward(ada.adaAttnHead[2 * i + 1], fcs, fs[i], fcs)
    return fcs, decoder_forward(ada.decoder, fcs)


def imagenet_normalize(x: torch.Tensor) -> torch.Tensor:
    """imageNet1k_normalize (vgg19.py:6-12)."""
    x = x.float()
    mean = x.new_tensor([0.485, 0.456, 0.406]).view(-1, 1, 1)
    std = x.new_tensor([0.229, 0.224, 0.225]).view(-1, 1, 1)
    return (x / 255.0 - mean) / std


def vgg19_forward(vgg, x: torch.Tensor, masked_features: bool = False) -> Dict[str, torch.Tensor]:
    """VGG19.forward (vgg19.py:42-70): relu1_1 .. relu5_1.  On a ROCm device: the HIP kernels
    (train_fns: zero-padded implicit-GEMM convs with fused ReLU, max-pool, fused normalise;
    features are NCHW views of NHWC storage); on the CPU: aten.  masked_features: see
    train_fns.vgg19_forward (the Trainer's fused feature losses)."""
    if x.is_cuda:
        from network.vgg19 import _CONVS, _POOLS, _SLICES
        from . import train_fns
        return train_fns.vgg19_forward(vgg, x, {i for i, _, _ in _CONVS}, set(_POOLS), _SLICES, masked_features)
    x = imagenet_normalize(x)
    feats = {}
    for i in range(1, 6):
        x = getattr(vgg, f"slice{i}")(x)
        feats[f"relu{i}_1"] = x
    return feats


def _tokens(x: torch.Tensor) -> torch.Tensor:
    """NCHW (any strides; free for channels-last views) -> contiguous fp32 [B][H*W][C]."""
    B, C, h, w = x.shape
    return x.permute(0, 2, 3, 1).float().contiguous().view(B, h * w, C)


def ada_attn_for_loss(c_x, s_x, c_1x, s_1x, activation: str = "softmax", chunk: int = 4096) -> torch.Tensor:
    """AdaAttnForLoss.forward (adaDecoder.py:52-81).  The training step needs it without gradients
    (its inputs are VGG features of the content and style images, lossfn.py:26-34): on a ROCm
    device that runs the wide-head HIP kernel (mhada_loss_attn: flash-style, A never stored,
    fp32 MFMA); the result is an NCHW view of token-major storage.  When a gradient is required
    (a caller differentiating through the target) or on the CPU, the reference expression is
    evaluated with aten ops, query-chunked so the Nc x Ns matrix is never whole."""
    grad = torch.is_grad_enabled() and any(t.requires_grad for t in (c_x, s_x, c_1x, s_1x))
    if c_x.is_cuda and not grad:
        from ._lib import ACT_COSINE, ACT_SOFTMAX
        unit = activation == "cosine"
        qt, kt, vt, xt = _tokens(c_1x), _tokens(s_1x), _tokens(s_x), _tokens(c_x)
        qn = ops.rows_normalize(qt, *ops.instnorm_stats(qt), unit=unit)
        kn = ops.rows_normalize(kt, *ops.instnorm_stats(kt), unit=unit)
        x_mu, x_rs = ops.instnorm_stats(xt)
        out = ops.loss_attn(qn, kn, vt, xt, x_mu, x_rs, ACT_COSINE if unit else ACT_SOFTMAX)
        B, C, h, w = c_x.shape
        return out.view(B, h, w, C).permute(0, 3, 1, 2)
    b, _, h, w = c_1x.shape
    q = F.instance_norm(c_1x).reshape(b, -1, h * w).permute(0, 2, 1)
    k = F.instance_norm(s_1x).reshape(b, s_1x.shape[1], -1)
    v = s_x.reshape(b, s_x.shape[1], -1).permute(0, 2, 1)
    ms, ss = [], []
    for q0 in range(0, q.shape[1], chunk):
        a = _softmax_or_cosine(q[:, q0:q0 + chunk], k, activation)
        m = torch.bmm(a, v)
        ms.append(m)
        ss.append(torch.sqrt((torch.bmm(a, v * v) - m * m).clamp(min=1e-6)))
    bc, _, hc, wc = c_x.shape
    m = torch.cat(ms, 1).reshape(bc, hc, wc, -1).permute(0, 3, 1, 2)
    s = torch.cat(ss, 1).reshape(bc, hc, wc, -1).permute(0, 3, 1, 2)
    return s * F.instance_norm(c_x) + m
