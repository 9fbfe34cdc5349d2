"""Winograd weight-gradient kernel (mhada_conv3x3_wgrad_wino) at the training step's decoder shapes
(the three AdaFormer calls batched: 24 images at 512^2): HIP-event median per call.  The round-5
A/B against the previous kernel (built with it as tuning xknob = 2) is profiles/r05_wgrad_ab.log.

    python tools/wgrad_ab.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch  # noqa: E402

from mhada_hip import ops  # noqa: E402
from opbench import bench  # noqa: E402


def main():
    for B, H, Ci, Co in ((24, 64, 512, 256), (24, 128, 256, 256), (24, 128, 256, 128), (24, 256, 128, 128),
                         (24, 256, 128, 64), (24, 512, 64, 64)):
        x = torch.randn(B, H, H, Ci, device="cuda")
        g = torch.randn(B, H, H, Co, device="cuda")
        fns = {"wgrad": lambda: ops.conv3x3_wgrad_wino(x, g, Co, "reflect", bias=True)}
        t = bench(fns, rounds=5, iters=3)
        fl = 2 * B * H * H * 9 * Ci * Co
        print(f"wgrad {Ci:3d}->{Co:3d} @{H:4d} B{B}: " + "  ".join(f"{k} {v * 1e3:8.1f} us {fl / v / 1e9:6.1f} TF(direct)"
                                                             for k, v in t.items()), flush=True)


if __name__ == "__main__":
    main()
