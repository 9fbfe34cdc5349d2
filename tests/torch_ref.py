"""Plain-PyTorch restatement of the forward path, used by the GPU tests as the full-size
floating-point reference (fp32 or fp64 on the device).  Test infrastructure only — it is
never imported by the product package.  Mirrors oracle/mhada_oracle.py (which is pinned to
the reference goldens); the small-size GPU tests compare against those goldens directly.
"""
import math

import torch
import torch.nn.functional as F


def vit(x, sd, heads=8, layers=3):
    """VisionTransformer.forward (vit.py:148-169), batch-axis attention (vit.py:59)."""
    B, _, H, W = x.shape
    h, w = H // 8, W // 8
    t = F.conv2d(x, sd["patch_embedding.conv_proj.weight"], sd["patch_embedding.conv_proj.bias"], stride=8)
    C = t.shape[1]
    t = t.reshape(B, C, h * w).permute(0, 2, 1)
    if "pos_embedding.pos_embed" in sd:
        pe = sd["pos_embedding.pos_embed"]
        if (h, w) != tuple(pe.shape[2:]):
            pe = F.interpolate(pe, size=(h, w), mode="bilinear", align_corners=False)
        t = t + pe.reshape(1, C, h * w).permute(0, 2, 1)
    outs = []
    d = C // heads
    for i in range(layers):
        p = f"encoder.{i}."
        y = F.layer_norm(t, (C,), sd[p + "ln1.weight"], sd[p + "ln1.bias"], 1e-6)
        qkv = F.linear(y, sd[p + "attention.in_proj_weight"], sd[p + "attention.in_proj_bias"])
        q, k, v = qkv.split(C, dim=-1)
        # (L=B, N, H, d) -> (N, H, L, d)
        q, k, v = (z.reshape(B, h * w, heads, d).permute(1, 2, 0, 3) for z in (q, k, v))
        a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d), dim=-1) @ v
        a = a.permute(2, 0, 1, 3).reshape(B, h * w, C)
        t = t + F.linear(a, sd[p + "attention.out_proj.weight"], sd[p + "attention.out_proj.bias"])
        y = F.layer_norm(t, (C,), sd[p + "ln2.weight"], sd[p + "ln2.bias"], 1e-6)
        y = F.linear(F.relu(F.linear(y, sd[p + "mlp.0.weight"], sd[p + "mlp.0.bias"])),
                     sd[p + "mlp.2.weight"], sd[p + "mlp.2.bias"])
        t = t + y
        outs.append(t.permute(0, 2, 1).reshape(B, C, h, w))
    return outs


def inorm(x, eps=1e-5):
    return F.instance_norm(x, eps=eps)


def block(fc, fs, fcs, sd, pre, heads=8, activation="softmax", chunk=4096):
    """AdaAttnMultiHead.forward (adaDecoder.py:162-206), query-chunked to bound memory."""
    B, C, h, w = fc.shape
    d = C // heads
    outs = []
    for i in range(heads):
        sl = slice(i * d, (i + 1) * d)
        q = F.conv2d(inorm(fc[:, sl]), sd[f"{pre}f_list.{i}.weight"], sd[f"{pre}f_list.{i}.bias"])
        k = F.conv2d(inorm(fs[:, sl]), sd[f"{pre}g_list.{i}.weight"], sd[f"{pre}g_list.{i}.bias"])
        v = F.conv2d(fs[:, sl], sd[f"{pre}h_list.{i}.weight"], sd[f"{pre}h_list.{i}.bias"])
        q = q.reshape(B, d, -1).permute(0, 2, 1)
        k = k.reshape(B, d, -1)
        v = v.reshape(B, d, -1).permute(0, 2, 1)
        ms, ss = [], []
        for c0 in range(0, q.shape[1], chunk):
            qq = q[:, c0:c0 + chunk]
            if activation == "softmax":
                a = torch.softmax(qq @ k, dim=-1)
            else:
                s = (qq @ k) / (qq.norm(dim=-1, keepdim=True) @ k.norm(dim=1, keepdim=True)) + 1
                a = s / s.sum(dim=-1, keepdim=True)
            m = a @ v
            var = a @ (v * v) - m * m
            ms.append(m)
            ss.append(torch.sqrt(var.clamp(min=1e-6)))
        m = torch.cat(ms, 1).reshape(B, h, w, d).permute(0, 3, 1, 2)
        s = torch.cat(ss, 1).reshape(B, h, w, d).permute(0, 3, 1, 2)
        outs.append(s * inorm(fcs[:, sl]) + m)
    return F.conv2d(torch.cat(outs, 1), sd[f"{pre}out_conv.weight"], sd[f"{pre}out_conv.bias"])


DEC = [("conv1.0", True), ("conv1.1", False), ("conv1.2", False), ("conv1.3", False), ("conv1.4", True),
       ("conv2.0", False), ("conv2.1", True), ("conv3.0", False), ("conv3.1", False)]


def decoder(x, sd, pre="decoder."):
    """Decoder.forward (conv.py:96-100)."""
    for name, up in DEC:
        x = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), sd[f"{pre}{name}.conv.conv.weight"],
                     sd[f"{pre}{name}.conv.conv.bias"])
        x = F.relu(x)
        if up:
            x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    return x


def adaformer(fc, fs, sd, activation="softmax"):
    fcs = fc[0]
    for i in range(3):
        fcs = block(fc[i], fs[i], fcs, sd, f"adaAttnHead.{2 * i}.", activation=activation)
        fcs = block(fcs, fs[i], fcs, sd, f"adaAttnHead.{2 * i + 1}.", activation=activation)
    return fcs, decoder(fcs, sd)


def stylize(c, s, sd_vc, sd_vs, sd_ada, activation="softmax"):
    fc = vit(c, sd_vc)
    fs = vit(s, sd_vs)
    fcs, cs = adaformer(fc, fs, sd_ada, activation)
    return fc, fs, fcs, cs
