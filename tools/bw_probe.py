"""HBM rate calibration on the box: torch copy / add against the repo's streaming kernels
(upsample2x, layernorm, residual GEMM) at the 1024^2 B4 decoder / ViT sizes."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops


def t(f, n=10):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); f(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return sorted(ts)[n // 2]


def rep(name, us, nbytes):
    print(f"{name:40s} {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)


x = torch.rand(4, 1024, 1024, 64, device="cuda").bfloat16()      # 537 MB
y = torch.empty_like(x)
rep("torch copy bf16 537MB", t(lambda: y.copy_(x)), 2 * x.numel() * 2)
a = torch.rand(65536 * 512, device="cuda"); b = torch.rand_like(a); c = torch.empty_like(a)
rep("torch add f32 3x134MB", t(lambda: torch.add(a, b, out=c)), 3 * a.numel() * 4)
xs = torch.rand(4, 512, 512, 64, device="cuda").bfloat16()
rep("upsample2x bf16 512->1024 x64", t(lambda: ops.upsample2x(xs)), xs.numel() * 2 * 5)
rep("torch interpolate (channels_last bf16)", t(lambda: torch.nn.functional.interpolate(
    xs.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear", align_corners=False)), xs.numel() * 2 * 5)
h = torch.rand(65536, 512, device="cuda")
g = torch.rand(512, device="cuda"); bb = torch.rand(512, device="cuda")
rep("layernorm f32->bf16 65536x512", t(lambda: ops.layernorm(h, g, bb, torch.bfloat16, 1e-6)), h.numel() * 6)
xb = torch.rand(65536, 512, device="cuda").bfloat16(); w = (torch.randn(512, 512, device="cuda") / 22).bfloat16()
bias = torch.rand(512, device="cuda"); r = torch.rand(65536, 512, device="cuda")
rep("residual GEMM 65536x512x512 f32 out", t(lambda: ops.linear(xb, w, bias, torch.float32, residual=r)),
    xb.numel() * 2 + 2 * r.numel() * 4)
