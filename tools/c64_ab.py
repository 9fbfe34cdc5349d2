"""bf16 decoder conv3.0 (64 -> 64 at 1024^2 B4, bilinear x2 of a 512^2 input): the direct tile
kernel with the upsample fused (conv3x3_c64 up=1) against upsample2x + the same kernel without
it (up=0), and the bits of both.   python tools/c64_ab.py"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops

B, H = 4, 512
x = torch.rand(B, H, H, 64, device="cuda").bfloat16()
w = (torch.randn(64, 9 * 64, device="cuda") / 24).bfloat16()
b = torch.randn(64, device="cuda")
fused = lambda: ops.conv3x3(x, w, b, torch.bfloat16, upsample=True)  # noqa: E731
split = lambda: ops.conv3x3(ops.upsample2x(x), w, b, torch.bfloat16, upsample=False)  # noqa: E731
ups = lambda: ops.upsample2x(x)  # noqa: E731
u = ops.upsample2x(x)
plain = lambda: ops.conv3x3(u, w, b, torch.bfloat16, upsample=False)  # noqa: E731
print("bit-identical:", torch.equal(fused(), split()))
res = {k: [] for k in ("fused", "split", "upsample", "conv_noup")}
for _ in range(9):
    for k, f in (("fused", fused), ("split", split), ("upsample", ups), ("conv_noup", plain)):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            f()
        e.record()
        torch.cuda.synchronize()
        res[k].append(s.elapsed_time(e) * 1e3 / 5)
fl = 2 * 9 * 64 * 64 * B * (2 * H) ** 2
for k, v in res.items():
    m = sorted(v)[4]
    print(f"{k:10s} {m:8.1f} us  {fl / m / 1e6:7.1f} TF/s (conv FLOPs)")
