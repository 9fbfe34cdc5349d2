"""The fp32 Winograd conv alone on one shape, a few launches (a target for rocprofv3 PMC passes).
    python tools/wino_only.py [B H Ci Co]   (default 8 128 256 256)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import _lib, ops

B, H, Ci, Co = map(int, sys.argv[1:5]) if len(sys.argv) > 4 else (8, 128, 256, 256)
x = torch.rand(B, H, H, Ci, device="cuda")
w = torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5
u = ops.wino_weights(w)
for _ in range(int(os.environ.get("ITERS", "5"))):
    ops.conv3x3_wino(x, u, None, True, "reflect", 1)
torch.cuda.synchronize()
print("done")
