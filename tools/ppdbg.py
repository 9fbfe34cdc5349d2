"""Ping-pong GEMM breakdown: time the kernel with DMA / LDS reads / barriers knocked out."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops
sys.path.insert(0, os.path.join(REPO, "tools"))
from opbench import bench, with_env

M = 65536
for N, K in ((512, 2048), (1536, 512)):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    fns = {f"dbg{d}": (lambda d=d: with_env("MHADA_GEMM_DBG", str(d), ops.linear, x, w, None, torch.bfloat16))
           for d in (0, 1, 2, 3, 4, 5, 6, 7)}
    t = bench(fns)
    fl = 2 * M * N * K
    print(f"N={N} K={K}: " + "  ".join(f"{k} {v * 1e3:6.1f}us {fl / v / 1e9:6.0f}TF" for k, v in t.items()))
