"""Interleaved-round A/B of bf16 MHAda attention (mhada_attn, the fsq kernel) tuning variants at the
configs[2] shape (1024^2 B4: Nc = Ns = 16384) or another, outputs compared bit for bit.

    S3_VARIANTS="base: il:xknob=1" python tools/attn_bf16_variants_interleaved.py [B Nc Ns rounds]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import _lib, ops


def main():
    B, Nc, Ns, rounds = (int(x) for x in (sys.argv[1:] + ["4", "16384", "16384", "11"][len(sys.argv) - 1:])[:4])
    variants = []
    for item in os.environ.get("S3_VARIANTS", "base:").split():
        name, _, kv = item.partition(":")
        variants.append((name, {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}))
    torch.manual_seed(0)
    H = 8
    q = (torch.randn(B, H, Nc, 64, device="cuda") * 0.5).to(torch.bfloat16)
    kv = (torch.randn(B, H, Ns, 128, device="cuda") * 0.5).to(torch.bfloat16)
    vt = ops.transpose_v(kv)
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
                for _ in range(3):
                    y = ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
                e.record()
                torch.cuda.synchronize()
            if r > 0:
                ts[name].append(s.elapsed_time(e) / 3)
            outs[name] = y
    base = outs[variants[0][0]]
    fl = 6.0 * Nc * Ns * 512 * B
    for name, _ in variants:
        t = sorted(ts[name])
        med = t[len(t) // 2]
        print(f"{name:8s} median {med:.4f} ms = {fl / med / 1e9 / 2500:.3f} of 2.5 PF (min {t[0]:.4f}, max {t[-1]:.4f})"
              f"  bit-identical to {variants[0][0]}: {torch.equal(outs[name], base)}", flush=True)


if __name__ == "__main__":
    main()
