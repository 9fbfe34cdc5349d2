"""Median time of the bf16 MHAda attention at 1024^2 B4 (HIP events).  usage: python tools/attn_time.py"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops
B, H, n = 4, 8, 16384
q = (torch.randn(B, H, n, 64, device="cuda") * 0.35).bfloat16()
kv = (torch.randn(B, H, n, 128, device="cuda") * 0.35).bfloat16()
vt = ops.transpose_v(kv)
fcs = torch.randn(B, n, 512, device="cuda")
mu, rs = ops.instnorm_stats(fcs)
vmu = torch.zeros(B, 512, device="cuda")
f = lambda: ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)  # noqa: E731
f()
ts = []
for _ in range(int(os.environ.get("ITERS", "10"))):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); f(); e.record(); torch.cuda.synchronize()
    ts.append(s.elapsed_time(e) * 1e3)
print(f"{sorted(ts)[len(ts) // 2]:.1f} us")
