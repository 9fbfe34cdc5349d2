"""Interleaved A/B of SPLIT3 attention tuning variants at one shape (default the 512^2 B8 bench shape):
every round times each variant once (in rotating order), medians over the rounds — the per-variant
blocks of tools/attn_s3_ab.py favour whichever variant runs later on a box that is still ramping up.

    S3_VARIANTS="base: il:xknob=1" python tools/attn_s3_variants_interleaved.py [B Nc Ns rounds]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import _lib, ops


def main():
    B, Nc, Ns, rounds = (int(x) for x in (sys.argv[1:] + ["8", "4096", "4096", "15"][len(sys.argv) - 1:])[:4])
    variants = []
    for item in os.environ.get("S3_VARIANTS", "base:").split():
        name, _, kv = item.partition(":")
        variants.append((name, {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}))
    torch.manual_seed(0)
    H = 8
    q = torch.randn(B, H, Nc, 64, device="cuda") * 0.5
    kv = torch.randn(B, H, Ns, 128, device="cuda") * 0.5
    img = ops.split3_kv(kv, ops.transpose_v(kv))
    fcs = torch.randn(B, Nc, 512, device="cuda")
    mu, rs = ops.instnorm_stats(fcs)
    vmu = torch.zeros(B, 512, device="cuda")
    outs, ts = {}, {n: [] for n, _ in variants}
    for r in range(rounds + 1):
        order = variants[r % len(variants):] + variants[:r % len(variants)]
        for name, knobs in order:
            with _lib.tuning(**knobs):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    y = ops.attn_split3(q, img, Ns, fcs, mu, rs, vmu)
                e.record()
                torch.cuda.synchronize()
            if r > 0:
                ts[name].append(s.elapsed_time(e) / 5)
            outs[name] = y
    base = outs[variants[0][0]]
    for name, _ in variants:
        t = sorted(ts[name])
        same = torch.equal(outs[name], base)
        print(f"{name:8s} median {t[len(t) // 2]:.4f} ms  (min {t[0]:.4f}, max {t[-1]:.4f})  bit-identical to "
              f"{variants[0][0]}: {same}", flush=True)


if __name__ == "__main__":
    main()
