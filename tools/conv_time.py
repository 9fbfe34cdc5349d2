"""Median time of one bf16 decoder conv shape (HIP events).  usage: python tools/conv_time.py Ci Co H up"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops

Ci, Co, H, up = map(int, sys.argv[1:5])
x = torch.rand(4, H, H, Ci, device="cuda").bfloat16()
w = (torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5).bfloat16()
b = torch.randn(Co, device="cuda")
f = lambda: ops.conv3x3(x, w, b, torch.bfloat16, upsample=bool(up))  # noqa: E731
f()
ts = []
for _ in range(int(os.environ.get("ITERS", "10"))):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); f(); e.record(); torch.cuda.synchronize()
    ts.append(s.elapsed_time(e) * 1e3)
print(f"{sorted(ts)[len(ts) // 2]:.1f} us")
