"""Interleaved-round A/B of the SPLIT3 training attention forward (ops.attn_train_fwd with TRAIN_FWD_S3) at
the 512^2 B8 step's shape (BH = 192, Nc = Ns = 4096) under tuning-knob variants; outputs compared bit
for bit.

    S3_VARIANTS="base: il:xknob=1" python tools/train_fwd_knob_ab.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import _lib, ops


def main():
    variants = []
    for item in os.environ.get("S3_VARIANTS", "base:").split():
        name, _, kv = item.partition(":")
        variants.append((name, {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}))
    torch.manual_seed(0)
    BH, n = 192, 4096
    q, k, v, x = (torch.randn(BH, n, 64, device="cuda") * 0.4 for _ in range(4))
    v = (v - v.mean(dim=1, keepdim=True)).contiguous()
    outs, ts = {}, {nm: [] for nm, _ in variants}
    for r in range(12):
        order = variants[r % len(variants):] + variants[:r % len(variants)]
        for name, knobs in order:
            with _lib.tuning(**knobs):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(2):
                    o = ops.attn_train_fwd(q, k, v, x)
                e.record()
                torch.cuda.synchronize()
            if r > 0:
                ts[name].append(s.elapsed_time(e) / 2)
            outs[name] = o
    b = outs[variants[0][0]]
    for name, _ in variants:
        t = sorted(ts[name])
        same = all(torch.equal(a, c) for a, c in zip(outs[name], b))
        print(f"{name:8s} median {t[len(t) // 2]:.3f} ms (min {t[0]:.3f}, max {t[-1]:.3f})  bit-identical: {same}",
              flush=True)


if __name__ == "__main__":
    main()
