"""fp32 GEMM/conv tile-shape A/B (MHADA_GEMM_F32_TILE), headline shapes (512^2 batch 8)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd"), os.path.join(REPO, "tools")]
import torch
from mhada_hip import ops
from opbench import bench, with_env

M = 32768
for (N, K, res) in [(1536, 512, False), (2048, 512, False), (512, 2048, True), (512, 512, True)]:
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda") if res else None
    fns = {t: (lambda t=t: with_env("MHADA_GEMM_F32_TILE", t, ops.linear, x, w, b, torch.float32, residual=r))
           for t in ("128x128", "256x128", "128x256")}
    ref = ops.linear(x, w, b, torch.float32, residual=r)
    for t, f in fns.items():
        assert torch.allclose(f(), ref, rtol=1e-4, atol=1e-4), t
    tm = bench(fns)
    fl = 2 * M * N * K
    print(f"gemm f32 N={N} K={K}: " + "  ".join(f"{k} {v * 1e3:6.1f}us {fl / v / 1e9:6.1f}TF" for k, v in tm.items()))
B = 8
for (Ci, Co, H) in [(512, 256, 64), (256, 256, 128), (256, 128, 128), (128, 128, 256), (128, 64, 256), (64, 64, 512)]:
    x = torch.rand(B, H, H, Ci, device="cuda")
    w = torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5
    bias = torch.randn(Co, device="cuda")
    fns = {t: (lambda t=t: with_env("MHADA_GEMM_F32_TILE", t, ops.conv3x3, x, w, bias, torch.float32))
           for t in ("128x128", "256x128", "128x256")}
    tm = bench(fns)
    fl = 2 * B * H * H * Co * 9 * Ci
    print(f"conv f32 {Ci}->{Co} @{H}: " + "  ".join(f"{k} {v * 1e3:7.1f}us {fl / v / 1e9:6.1f}TF" for k, v in tm.items()))
