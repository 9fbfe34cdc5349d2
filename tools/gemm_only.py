"""Run one GEMM shape a few times (for rocprofv3 PMC passes).
usage: python tools/gemm_only.py f32|bf16 M N K [res]"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops

dt = torch.bfloat16 if sys.argv[1] == "bf16" else torch.float32
M, N, K = map(int, sys.argv[2:5])
res = len(sys.argv) > 5 and sys.argv[5] == "res"
x = torch.randn(M, K, device="cuda").to(dt)
w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
b = torch.randn(N, device="cuda")
r = torch.randn(M, N, device="cuda") if res else None
for _ in range(int(os.environ.get("ITERS", "5"))):
    ops.linear(x, w, b, torch.float32 if res else dt, residual=r)
torch.cuda.synchronize()
print("done")
