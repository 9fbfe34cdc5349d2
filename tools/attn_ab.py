"""A/B of the bf16 MHAda attention kernel variants (attn_* tuning knobs, attn.hip) in one process:
agreement on the same operands and interleaved timing (median of rounds) at the bench shapes.

    python tools/attn_ab.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch

from mhada_hip import ops

SHAPES = [("1024^2 B4", 4, 16384, 16384), ("512^2 B8", 8, 4096, 4096), ("video 1080p/s256", 1, 32400, 1024),
          ("ragged", 2, 1000, 777)]


VARIANTS = {"fsq1P0": {"attn_fixed_shift": 1, "attn_prio": 0},
            "fsq1": {"attn_fixed_shift": 1, "attn_prio": 1},
            "w8": {"attn_fixed_shift": 0, "attn_tk": 128}}


def run(variant, args):
    from mhada_hip import _lib
    with _lib.tuning(**VARIANTS[variant]):
        return ops.mhada_attn(*args, 0)


def main():
    torch.manual_seed(0)
    H = 8
    for name, B, nc, ns in SHAPES:
        q = (torch.randn(B, H, nc, 64, device="cuda") * 0.35).bfloat16()
        kv = (torch.randn(B, H, ns, 128, device="cuda") * 0.35).bfloat16()
        vt = ops.transpose_v(kv)
        fcs = torch.randn(B, nc, 512, device="cuda")
        mu, rs = ops.instnorm_stats(fcs)
        vmu = torch.zeros(B, 512, device="cuda")
        args = (q, kv, vt, fcs, mu, rs, vmu)
        ref = run("w8", args).float()
        errs = {v: ((run(v, args).float() - ref).abs().max() / ref.abs().max()).item() for v in VARIANTS}
        times = {v: [] for v in VARIANTS}
        for _ in range(7):
            for v in VARIANTS:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    run(v, args)
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / 5)
        med = {k: sorted(v)[3] for k, v in times.items()}
        fl = 6.0 * nc * ns * 512 * B
        print(f"{name:18s} " + "   ".join(f"{v} {med[v]:.3f} ms {fl / med[v] / 1e9:.0f} TF (err {errs[v]:.1e})"
                                           for v in VARIANTS), flush=True)
    # fp32 (one kernel; compare with the launch averages in profiles/r01_attn_launch_stats.txt)
    if os.environ.get("ATTN_AB_NO_F32"):
        return
    for name, B, nc, ns in SHAPES[1:]:
        q = torch.randn(B, H, nc, 64, device="cuda") * 0.35
        kv = torch.randn(B, H, ns, 128, device="cuda") * 0.35
        vt = ops.transpose_v(kv)
        fcs = torch.randn(B, nc, 512, device="cuda")
        mu, rs = ops.instnorm_stats(fcs)
        vmu = torch.zeros(B, 512, device="cuda")
        ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 3)
        t = sorted(ts)[3]
        print(f"fp32 {name:18s} {t:.3f} ms {6.0 * nc * ns * 512 * B / t / 1e9:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
