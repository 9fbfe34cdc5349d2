"""fp32 3x3 conv: Winograd F(2x2,3x3) (wino.hip) vs the direct implicit GEMM, median HIP-event
time per shape.  usage: python tools/wino_ab.py [iters]"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
# (name, B, H, Ci, Co, pad_mode, pad): 512^2 B8 decoder layers, VGG19 at 512^2 B8, a dgrad shape
SHAPES = [("dec1 512->256 @64", 8, 64, 512, 256, "reflect", 1), ("dec2 256->256 @128", 8, 128, 256, 256, "reflect", 1),
          ("dec5 256->128 @128", 8, 128, 256, 128, "reflect", 1), ("dec6 128->128 @256", 8, 256, 128, 128, "reflect", 1),
          ("dec7 128->64 @256", 8, 256, 128, 64, "reflect", 1), ("dec8 64->64 @512", 8, 512, 64, 64, "reflect", 1),
          ("vgg1_2 64->64 @512", 8, 512, 64, 64, "zero", 1), ("vgg2_2 128->128 @256", 8, 256, 128, 128, "zero", 1),
          ("vgg3 256->256 @128", 8, 128, 256, 256, "zero", 1), ("vgg4 512->512 @64", 8, 64, 512, 512, "zero", 1),
          ("dgrad 256->256 @128 pad2", 8, 128, 256, 256, "zero", 2)]


def med(f):
    f()
    ts = []
    for _ in range(ITERS):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); f(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return sorted(ts)[len(ts) // 2]


for name, B, H, Ci, Co, pm, pad in SHAPES:
    x = torch.rand(B, H, H, Ci, device="cuda")
    w = torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5
    b = torch.randn(Co, device="cuda")
    u = ops.wino_weights(w)
    Ho = H + 2 * (pad - 1)
    flop = 2.0 * 9 * Ci * Co * B * Ho * Ho
    tw = med(lambda: ops.conv3x3_wino(x, u, b, True, pm, pad))
    ops.WINO = False
    td = med(lambda: ops.conv3x3(x, w, b, torch.float32, upsample=False, relu=True, pad_mode=pm, pad=pad))
    ops.WINO = True
    err = (ops.conv3x3_wino(x, u, b, True, pm, pad) - ops.conv3x3(x, w, b, torch.float32, upsample=False,
                                                                 pad_mode=pm, pad=pad)).abs().max().item()
    print(f"{name:26s} wino {tw:8.1f} us ({flop / tw / 1e6:6.1f} direct-equiv TF/s, {flop / 2.25 / tw / 1e6:6.1f} TF/s "
          f"MFMA)  direct {td:8.1f} us ({flop / td / 1e6:6.1f} TF/s)  x{td / tw:.2f}  max|d|={err:.2e}", flush=True)
