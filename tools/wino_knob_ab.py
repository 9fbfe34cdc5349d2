"""fp32 Winograd conv tuning knobs A/B in one process (interleaved rounds, median), at the 512^2 B8
decoder / VGG19 / dgrad shapes.   python tools/wino_knob_ab.py <knob> [iters]   (e.g. wino_l2pf)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import _lib, ops

KNOB = sys.argv[1]
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
SHAPES = [("dec1 512->256 @64", 8, 64, 512, 256, "reflect", 1), ("dec2 256->256 @128", 8, 128, 256, 256, "reflect", 1),
          ("dec5 256->128 @128", 8, 128, 256, 128, "reflect", 1), ("dec6 128->128 @256", 8, 256, 128, 128, "reflect", 1),
          ("dec7 128->64 @256", 8, 256, 128, 64, "reflect", 1), ("vgg1_2 64->64 @512", 8, 512, 64, 64, "zero", 1),
          ("vgg2_2 128->128 @256", 8, 256, 128, 128, "zero", 1), ("vgg3 256->256 @128", 8, 128, 256, 256, "zero", 1),
          ("vgg4 512->512 @64", 8, 64, 512, 512, "zero", 1), ("dgrad 256->256 @128 pad2", 8, 128, 256, 256, "zero", 2)]


def timed(f):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(ITERS):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / ITERS


tot = {0: 0.0, 1: 0.0}
for name, B, H, Ci, Co, pm, pad in SHAPES:
    x = torch.rand(B, H, H, Ci, device="cuda")
    w = torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5
    b = torch.randn(Co, device="cuda")
    u = ops.wino_weights(w)
    f = lambda: ops.conv3x3_wino(x, u, b, True, pm, pad)  # noqa: E731
    outs, ts = {}, {0: [], 1: []}
    for v in (0, 1):
        with _lib.tuning(**{KNOB: v}):
            outs[v] = f().clone()
    for _ in range(7):
        for v in (0, 1):
            with _lib.tuning(**{KNOB: v}):
                ts[v].append(timed(f))
    m = {v: sorted(t)[3] for v, t in ts.items()}
    for v in (0, 1):
        tot[v] += m[v]
    print(f"{name:28s} {KNOB}=0 {m[0]:8.1f} us   {KNOB}=1 {m[1]:8.1f} us   1/0 {m[1] / m[0]:.3f}   "
          f"bit-identical {torch.equal(outs[0], outs[1])}", flush=True)
print(f"sum of medians: 0 {tot[0]:.1f} us, 1 {tot[1]:.1f} us ({tot[1] / tot[0]:.3f})")
