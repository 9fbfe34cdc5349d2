"""fp32 Winograd conv tuning knobs A/B in one process (interleaved rounds, median), at the 512^2 B8
decoder / VGG19 / dgrad shapes.
    python tools/wino_knob_ab.py <knob> [iters]                  (knob = 0 vs 1, e.g. xknob)
    python tools/wino_knob_ab.py -c xknob=0 -c xknob=1 ... [iters]   (any settings)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import _lib, ops

args = sys.argv[1:]
CFGS = []
while "-c" in args:
    i = args.index("-c")
    CFGS.append(dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in args[i + 1].split(",")))
    del args[i:i + 2]
if not CFGS:
    knob = args.pop(0)
    CFGS = [{knob: 0}, {knob: 1}]
ITERS = int(args[0]) if args else 5
NAMES = [",".join(f"{k}={v}" for k, v in c.items()) for c in CFGS]
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


tot = [0.0] * len(CFGS)
for name, B, H, Ci, Co, pm, pad in SHAPES:
    x = torch.rand(B, H, H, Ci, device="cuda")
    w = torch.randn(Co, 9 * Ci, device="cuda") / (9 * Ci) ** 0.5
    b = torch.randn(Co, device="cuda")
    u = ops.wino_weights(w)
    f = lambda: ops.conv3x3_wino(x, u, b, True, pm, pad)  # noqa: E731
    outs, ts = [], [[] for _ in CFGS]
    for c in CFGS:
        with _lib.tuning(**c):
            outs.append(f().clone())
    for _ in range(7):
        for i, c in enumerate(CFGS):
            with _lib.tuning(**c):
                ts[i].append(timed(f))
    m = [sorted(t)[3] for t in ts]
    for i in range(len(CFGS)):
        tot[i] += m[i]
    same = all(torch.equal(outs[0], o) for o in outs[1:])
    print(f"{name:26s} " + "  ".join(f"[{n}] {v:7.1f} us ({v / m[0]:.3f})" for n, v in zip(NAMES, m)) +
          f"  bit-identical {same}", flush=True)
print("sum of medians: " + ", ".join(f"[{n}] {t:.1f} us ({t / tot[0]:.3f})" for n, t in zip(NAMES, tot)))
