"""Video-path helpers with the reference's signatures.

* ``warp(x, flo, padding_mode)`` — ``utilities.warp`` (utilities.py:100-118);
* ``flow_warp_mask(flo01, flo10, padding_mode, threshold)`` — utilities.py:121-151;
* ``cv2_to_tensor(img, resize)`` — utilities.py:43-52 (BGR->RGB, INTER_AREA, toTensor255) as one
  HIP pass over the u8 frame in device memory (csrc/ingest.hip);
* ``warping_error(cs1, cs2, flow, mask)`` — the per-frame optical-flow metric of
  exps_sintel.py:101-109 (sum(mask * |cs2 - warp(cs1, flow)|) / (C*H*W));
* ``VideoStylizer`` — the infer_video.py:58-92 loop: the style is encoded once and, through the
  AdaFormer's per-style cache (engine.style_cache), its K/V projections are reused per frame.

The inference forms run the HIP kernels (csrc/warp.hip); the gradient through the warp w.r.t. the
image (train_video.py temporal losses) runs its HIP adjoint (WarpFn / mhada_warp_bwd).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import losses, ops


class WarpFn(torch.autograd.Function):
    """utilities.warp under autograd w.r.t. the image (train_video.py:147-151): forward mhada_warp,
    backward its adjoint mhada_warp_bwd.  The flow is data there (no gradient)."""

    @staticmethod
    def forward(ctx, x, flo, padding_mode):
        ctx.save_for_backward(flo)
        ctx.padding_mode = padding_mode
        return ops.warp(x, flo, padding_mode)

    @staticmethod
    def backward(ctx, gy):
        (flo,) = ctx.saved_tensors
        return ops.warp_bwd(gy, flo, ctx.padding_mode), None, None


def warp(x: torch.Tensor, flo: torch.Tensor, padding_mode: str = "zeros") -> torch.Tensor:
    """utilities.warp: bilinear backward warp of x [B,C,H,W] by flow flo [B,2,H,W].  On the device:
    the HIP kernel, with its HIP adjoint when x takes a gradient.  A flow that takes a gradient
    (no reference script differentiates through the flow) evaluates the reference expression with
    differentiable device ops (mhada_hip.losses.warp)."""
    if torch.is_grad_enabled() and flo.requires_grad:
        return losses.warp(x, flo, padding_mode)
    if torch.is_grad_enabled() and x.requires_grad:
        return WarpFn.apply(x, flo, padding_mode)
    return ops.warp(x, flo, padding_mode)


def cv2_to_tensor(img, resize: Optional[tuple] = None, device: Optional[torch.device] = None) -> torch.Tensor:
    """utilities.cv2_to_tensor: ``img`` is a cv2 BGR u8 frame (H, W, 3) — a numpy array (uploaded
    through pinned memory to ``device``, default the current ROCm device) or a uint8 device
    tensor; ``resize`` = (width, height) as cv2.resize takes it.  Returns the fp32 (3, h, w)
    tensor in [0, 255] on the device (the reference returns it on the CPU and moves it with
    .to(device) at infer_video.py:81).

    Shrinking uses INTER_AREA's box average; enlarging (any axis) OpenCV's area-mode 2-tap
    interpolation (csrc/ingest.hip), as cv2.resize(INTER_AREA) does — so a low-resolution video
    resized to a fixed IMAGE_SIZE (exps_video.py:84, infer_video.py:80) works as in the reference.
    cv2 is not installed here: parity with cv2's bits is unpinned."""
    if not isinstance(img, torch.Tensor):
        t = torch.from_numpy(img)
        if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
            raise ValueError("cv2_to_tensor expects a uint8 (H, W, 3) BGR frame")
        img = t.pin_memory().to(device or torch.device("cuda", torch.cuda.current_device()), non_blocking=True)
    out_hw = None if resize is None else (int(resize[1]), int(resize[0]))
    return ops.frame_ingest(img, out_hw, bgr=True)[0]


def flow_warp_mask(flo01: torch.Tensor, flo10: torch.Tensor, padding_mode: str = "zeros",
                   threshold: float = 2) -> torch.Tensor:
    """utilities.flow_warp_mask: forward/backward flow consistency mask [H,W] (1.0 = valid)."""
    return ops.flow_warp_mask(flo01, flo10, padding_mode, threshold)


def warping_error(cs1: torch.Tensor, cs2: torch.Tensor, flow: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """exps_sintel.py:101-109 per image: sum(mask * |cs2 - warp(cs1, flow)|) / (C*H*W).
    mask is [B,H,W] (or [H,W] for B == 1)."""
    if mask.dim() == 2:
        mask = mask.unsqueeze(0)
    return ops.warp_l1(cs1, cs2, flow, mask)


class VideoStylizer:
    """infer_video.py:58-92 on the drop-in modules: ``set_style(s)`` encodes the style once,
    ``__call__(frame)`` stylises one content frame [B,3,H,W] (0..255) against it and returns the
    clamped output; ``warping_error(flow, mask)`` scores the last two outputs (exps_sintel)."""

    def __init__(self, vit_c, vit_s, ada):
        self.vit_c, self.vit_s, self.ada = vit_c, vit_s, ada
        self.fs = None
        self.prev: Optional[torch.Tensor] = None
        self.cur: Optional[torch.Tensor] = None

    @torch.no_grad()
    def set_style(self, s: torch.Tensor) -> None:
        self.fs = self.vit_s(s)

    @torch.no_grad()
    def __call__(self, frame: torch.Tensor) -> torch.Tensor:
        if self.fs is None:
            raise RuntimeError("VideoStylizer: call set_style(style_image) first")
        _, cs = self.ada(self.vit_c(frame), self.fs)
        cs = cs.clamp(0, 255)
        self.prev, self.cur = self.cur, cs
        return cs

    @torch.no_grad()
    def warping_error(self, flow: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        if self.prev is None:
            raise RuntimeError("VideoStylizer: need two frames")
        return warping_error(self.prev / 255.0, self.cur / 255.0, flow, mask)
