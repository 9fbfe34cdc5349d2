"""Golden vectors for the video path's warp functions, produced by the
reference's own utilities.py / lossfn.py (imported with the stand-ins of make_train_goldens.py;
warp and flow_warp_mask use neither torchvision nor cv2).

Stored: inputs (images, flows) and the reference's outputs for
  * utilities.warp(x, flow, "zeros" | "border")          (utilities.py:100-118)
  * utilities.flow_warp_mask(flo01, flo10)                (utilities.py:121-151)
  * the exps_sintel.py:101-109 warping error of two frames
  * lossfn.output_level_temporal_loss / feature_level_temporal_loss (lossfn.py:50-86).
Flows reach +-7 px on a 20x33 image so every padding branch is taken.

Usage:  python tests/golden/make_video_goldens.py
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from make_train_goldens import load_reference, np32  # noqa: E402


def smooth_flow(g, B, H, W, amp):
    """Translation + low-frequency swirl + noise, [B, 2, H, W]."""
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    out = []
    for _ in range(B):
        t = (torch.rand(2, generator=g) - 0.5) * 2 * amp
        ph = torch.rand(2, generator=g) * 6.28
        fx = t[0] + 0.5 * amp * torch.sin(yy / 5.0 + ph[0]) + 0.3 * torch.randn(H, W, generator=g)
        fy = t[1] + 0.5 * amp * torch.cos(xx / 7.0 + ph[1]) + 0.3 * torch.randn(H, W, generator=g)
        out.append(torch.stack((fx, fy)))
    return torch.stack(out)


def main():
    ref = load_reference()
    U, L = ref["utilities"], ref["lossfn"]
    g = torch.Generator().manual_seed(20251015)
    B, C, H, W = 2, 3, 20, 33
    x = torch.rand(B, C, H, W, generator=g) * 255
    flow = smooth_flow(g, B, H, W, 5.0)
    out = {"x": np32(x), "flow": np32(flow),
           "warp_zeros": np32(U.warp(x, flow)), "warp_border": np32(U.warp(x, flow, padding_mode="border"))}
    # forward / backward flows: flo10 ~ -flo01 with noise so the mask is mixed
    flo01 = smooth_flow(g, 1, H, W, 4.0)[0]
    flo10 = -flo01 + 1.5 * torch.randn(2, H, W, generator=g)
    out.update(flo01=np32(flo01), flo10=np32(flo10), mask=np32(U.flow_warp_mask(flo01, flo10)))
    # exps_sintel.py:101-109 on two "stylised" frames in [0, 1]
    cs1 = torch.rand(1, 3, H, W, generator=g)
    cs2 = torch.rand(1, 3, H, W, generator=g)
    fl1 = flow[:1]
    m = torch.from_numpy(out["mask"]).unsqueeze(0)
    wc = U.warp(cs1, fl1)
    mk = m.unsqueeze(1).expand(-1, 3, -1, -1)
    err = torch.sum(mk * nn.L1Loss(reduction="none")(cs2, wc)) / (3 * H * W)
    out.update(cs1=np32(cs1), cs2=np32(cs2), warp_err=np.array(float(err)))
    # temporal losses (train_video.py uses MSELoss(reduction="none") as lossMatrix)
    c1 = torch.rand(1, 3, H, W, generator=g) * 255
    c2 = torch.rand(1, 3, H, W, generator=g) * 255
    mse = nn.MSELoss(reduction="none")
    out.update(c1=np32(c1), c2=np32(c2),
               out_temporal=np.array(float(L.output_level_temporal_loss(c1, c2, cs1 * 255, cs2 * 255, fl1, m, mse))))
    f1 = torch.randn(1, 8, 5, 9, generator=g)
    f2 = torch.randn(1, 8, 5, 9, generator=g)
    out.update(f1=np32(f1), f2=np32(f2),
               feat_temporal=np.array(float(L.feature_level_temporal_loss(f1, f2, fl1, m, mse))))
    path = os.path.join(HERE, "video_warp.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: mask mean {out['mask'].mean():.3f}, warp_err {float(err):.5f}, "
          f"out_temporal {float(out['out_temporal']):.3f}, feat_temporal {float(out['feat_temporal']):.4f}")


if __name__ == "__main__":
    main()
