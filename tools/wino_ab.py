"""A/B timing of the fp32 Winograd conv kernels (tuning wino4 0 / 1) on the decoder / VGG shapes
of the 512^2 batch-8 step and the training step, interleaved rounds in one process.

    python tools/wino_ab.py

Ablations of the 4-wave kernel (profiles/r05_wino4_ablate.log) come from builds with
-DWINO4_DBG=<mask> (1 no DMA, 2 no transform, 4 no MFMA, 8 no DMA wait; results invalid).
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd"), os.path.dirname(os.path.abspath(__file__))]

import torch

from mhada_hip import _lib, ops
from opbench import bench


def main():
    dev = "cuda"
    torch.manual_seed(0)
    for (B, H, Ci, Co, pad_mode) in [(8, 64, 512, 256, "reflect"), (8, 128, 256, 256, "reflect"),
                                     (8, 128, 256, 128, "reflect"), (8, 256, 128, 128, "reflect"),
                                     (8, 256, 128, 64, "reflect"), (8, 512, 64, 64, "reflect"),
                                     (8, 256, 64, 128, "zero"), (8, 128, 128, 256, "zero"), (8, 64, 256, 512, "zero")]:
        x = torch.randn(B, H, H, Ci, device=dev)
        w = torch.randn(Co, 9 * Ci, device=dev) / (9 * Ci) ** 0.5
        b = torch.randn(Co, device=dev)
        u = ops.wino_weights(w)
        out = torch.empty(B, H, H, Co, device=dev)

        def run(k):
            with _lib.tuning(wino4=k):
                ops.conv3x3_wino(x, u, b, True, pad_mode, 1, out=out)
        t = bench({"w8": lambda: run(0), "w4": lambda: run(1)})
        fl = 2 * B * H * H * Co * 9 * Ci / 2.25  # Winograd products
        print(f"wino {pad_mode:7s} B={B} {H:3d}^2 {Ci:3d}->{Co:3d}: " + "  ".join(
            f"{k} {v * 1e3:7.1f} us {fl / v / 1e9:6.1f} TF(wino)" for k, v in t.items()), flush=True)


if __name__ == "__main__":
    main()
