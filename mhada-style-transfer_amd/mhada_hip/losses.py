"""Training losses — restatement of ``MHAdaSTr/lossfn.py`` and the feature/flow utilities it
uses (``utilities.py:86-151``).  Same signatures as the reference functions."""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F


def feature_down_sample(feat: Dict[str, torch.Tensor], last_layer: int) -> torch.Tensor:
    """utilities.py:86-97"""
    size = feat[f"relu{last_layer}_1"].shape[-2:]
    parts = [F.interpolate(feat[f"relu{i}_1"], size=size, mode="bilinear", align_corners=False)
             for i in range(1, last_layer)]
    parts.append(feat[f"relu{last_layer}_1"])
    return torch.cat(parts, dim=1)


def global_style_loss(fcs, fs, loss_fn):
    """lossfn.py:7-23 — per-channel mean and UNBIASED std distances over relu1_1..relu5_1."""
    loss = 0
    for i in (1, 2, 3, 4, 5):
        a, b = fcs[f"relu{i}_1"], fs[f"relu{i}_1"]
        loss = loss + (loss_fn(a.mean(dim=(2, 3)), b.mean(dim=(2, 3))) + loss_fn(a.std(dim=(2, 3)), b.std(dim=(2, 3))))
    return loss


def local_feature_loss(fc, fs, fcs, adaattn_no_learn, loss_fn):
    """lossfn.py:26-34"""
    loss = 0
    for idx, i in enumerate((3, 4, 5)):
        target = adaattn_no_learn[idx](fc[f"relu{i}_1"], fs[f"relu{i}_1"], feature_down_sample(fc, i),
                                       feature_down_sample(fs, i))
        loss = loss + loss_fn(fcs[f"relu{i}_1"], target)
    return loss


def identity_loss_1(cc, c, ss, s, loss_fn):
    """lossfn.py:37-38"""
    return loss_fn(cc, c) + loss_fn(ss, s)


def identity_loss_2(fcc, fc, fss, fs, loss_fn):
    """lossfn.py:41-47"""
    loss = 0
    for i in (1, 2, 3, 4, 5):
        loss = loss + loss_fn(fcc[f"relu{i}_1"], fc[f"relu{i}_1"]) + loss_fn(fss[f"relu{i}_1"], fs[f"relu{i}_1"])
    return loss


def warp(x: torch.Tensor, flo: torch.Tensor, padding_mode: str = "zeros") -> torch.Tensor:
    """utilities.py:100-118.  NB the reference normalises the grid with (W-1) but samples with
    align_corners=False; reproduced as is."""
    B, C, H, W = x.shape
    yy, xx = torch.meshgrid(torch.arange(H, device=x.device), torch.arange(W, device=x.device), indexing="ij")
    grid = torch.stack((xx, yy), 0).float().unsqueeze(0).expand(B, -1, -1, -1)
    vgrid = grid + flo
    gx = 2.0 * vgrid[:, 0] / max(W - 1, 1) - 1.0
    gy = 2.0 * vgrid[:, 1] / max(H - 1, 1) - 1.0
    return F.grid_sample(x, torch.stack((gx, gy), dim=-1), mode="bilinear", padding_mode=padding_mode,
                         align_corners=False)


def _warp(x: torch.Tensor, flo: torch.Tensor) -> torch.Tensor:
    """warp as the temporal losses call it: on a ROCm device the HIP kernel and its HIP adjoint
    (video.warp), on the CPU the reference expression above."""
    if x.is_cuda:
        from .video import warp as device_warp
        return device_warp(x, flo)
    return warp(x, flo)


def output_level_temporal_loss(c1, c2, cs1, cs2, flow, mask, loss_matrix):
    """lossfn.py:50-66"""
    input_term = c2 - _warp(c1, flow)
    input_term = 0.2126 * input_term[:, 0] + 0.7152 * input_term[:, 1] + 0.0722 * input_term[:, 2]
    input_term = input_term.unsqueeze(1).expand(-1, c2.shape[1], -1, -1)
    output_term = cs2 - _warp(cs1, flow)
    m = mask.unsqueeze(1).expand(-1, c2.shape[1], -1, -1)
    loss = torch.sum(m * loss_matrix(output_term, input_term))
    return loss * (1 / torch.nonzero(m).shape[0])


def feature_level_temporal_loss(f1, f2, flow, mask, loss_matrix):
    """lossfn.py:69-86"""
    feature_flow = F.interpolate(flow, size=f1.shape[2:], mode="bilinear")
    feature_flow[:, 0] *= float(f1.shape[3]) / flow.shape[3]
    feature_flow[:, 1] *= float(f1.shape[2]) / flow.shape[2]
    warped = _warp(f1, feature_flow)
    fm = F.interpolate(mask.unsqueeze(1), size=f1.shape[2:], mode="bilinear").squeeze(1)
    fm = (fm > 0).float().unsqueeze(1).expand(-1, f1.shape[1], -1, -1)
    loss = torch.sum(fm * loss_matrix(f2, warped))
    return loss * (1 / torch.nonzero(fm).shape[0])
