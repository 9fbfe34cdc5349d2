"""Run one bf16 decoder conv shape a few times (for rocprofv3 PMC passes).
usage: python tools/conv_only.py Ci Co H up   (H = input size; batch 4)"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops

Ci, Co, H, up = map(int, sys.argv[1:5])
x = torch.rand(4, H, H, Ci, device="cuda").bfloat16()
w = (torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5).bfloat16()
b = torch.randn(Co, device="cuda")
for _ in range(int(os.environ.get("ITERS", "5"))):
    ops.conv3x3(x, w, b, torch.bfloat16, upsample=bool(up))
torch.cuda.synchronize()
print("done")
