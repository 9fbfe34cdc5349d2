"""Probe for DESIGN §7.5: fp32-accurate GEMM products on the bf16 MFMA pipe.  Each fp32 operand is
split into three bf16 terms (x = x1 + x2 + x3, 8 mantissa bits each) and the six significant cross
products are summed in fp32 by ONE bf16 GEMM over the concatenated K axis:
    A' = [a2 | a3 | a1 | a2 | a1 | a1],  W' = [w2 | w1 | w3 | w1 | w2 | w1]   (small terms first)
Prints, at the fp32 headline's GEMM shapes, the error against fp64 of this form and of the native
fp32 GEMM (mhada_gemm fp32), and the time of the K' = 6K bf16 GEMM alone (the split itself would be
fused into the producers).  Not a product path: a measurement for the next round's design.

    python tools/split_bf16_probe.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch

from mhada_hip import ops


def split3(x):
    x1 = x.bfloat16()
    r = x - x1.float()
    x2 = r.bfloat16()
    x3 = (r - x2.float()).bfloat16()
    return x1, x2, x3


def timed(f, n=10):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            f()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / n * 1e3)
    return sorted(ts)[2]


def rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


def main():
    torch.manual_seed(0)
    M = 32768
    for N, K in ((1536, 512), (2048, 512), (512, 2048), (512, 512)):
        a = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") / K ** 0.5
        a1, a2, a3 = split3(a)
        w1, w2, w3 = split3(w)
        ap = torch.cat([a2, a3, a1, a2, a1, a1], dim=1).contiguous()
        wp = torch.cat([w2, w1, w3, w1, w2, w1], dim=1).contiguous()
        rows = torch.arange(0, M, 61, device="cuda")
        ref = a[rows].double() @ w.double().T
        y32 = ops.linear(a, w, None, torch.float32)
        ys = ops.linear(ap, wp, None, torch.float32)
        y16 = ops.linear(a.bfloat16(), w.bfloat16(), None, torch.float32)
        t32 = timed(lambda: ops.linear(a, w, None, torch.float32))
        ts = timed(lambda: ops.linear(ap, wp, None, torch.float32))
        fl = 2 * M * N * K
        print(f"M={M} N={N:5d} K={K:5d}: fp32 GEMM {t32:7.1f} us ({fl / t32 / 1e6:6.1f} TF) err {rel(y32[rows], ref):.2e} | "
              f"split-bf16 x6 (K'={6 * K}) {ts:7.1f} us ({fl / ts / 1e6:6.1f} fp32-TF) err {rel(ys[rows], ref):.2e} | "
              f"plain bf16 err {rel(y16[rows], ref):.2e}", flush=True)


if __name__ == "__main__":
    main()
