"""Cost of the SPLIT3 GEMM's output forms at the 512^2 B8 MLP1 shape (M = 32768, N = 2048, K0 = 512,
bias + ReLU): fp32 C only, the three bf16 planes only (inference: MLP1 -> MLP2), both (training hand-off);
and the QKV shape (N = 1536, fp32 C) for reference.  Interleaved rounds, median.

    python tools/split3_epilogue_ab.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import ops


def timeit(fn, iters=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    torch.manual_seed(0)
    M, C = 32768, 512
    planes = ops.split3_rows(torch.randn(M, C, device="cuda"))
    w1 = ops.split3_weight(torch.randn(4 * C, C, device="cuda") * C ** -0.5)
    wq = ops.split3_weight(torch.randn(3 * C, C, device="cuda") * C ** -0.5)
    b4, b3 = torch.zeros(4 * C, device="cuda"), torch.zeros(3 * C, device="cuda")
    variants = {
        "mlp1 fp32 C": lambda: ops.linear_split3(planes, w1, b4, torch.float32, relu=True),
        "mlp1 planes": lambda: ops.linear_split3(planes, w1, b4, torch.float32, relu=True, out_planes=True),
        "mlp1 both": lambda: ops.linear_split3(planes, w1, b4, torch.float32, relu=True, both=True),
        "qkv fp32 C": lambda: ops.linear_split3(planes, wq, b3, torch.float32),
    }
    for f in variants.values():
        f()
    torch.cuda.synchronize()
    ts = {k: [] for k in variants}
    for _ in range(7):
        for k, f in variants.items():
            ts[k].append(timeit(f))
    for k, v in ts.items():
        v.sort()
        print(f"{k:14s} median {v[len(v) // 2]:7.1f} us  (min {v[0]:.1f}, max {v[-1]:.1f})", flush=True)


if __name__ == "__main__":
    main()
