"""A/B of the training backward's dQ = dS K at the 512^2 B8 step's shape (BH = 192, Nc = Ns = 4096,
dS 12.9 GB): the fp32-MFMA N <= 64 GEMM (gemm_n64_kernel) against the SPLIT3 GEMM
(mhada_gemm_n64_split3, plus mhada_transpose64_split3 for its K^T planes), interleaved rounds, median; error of each
against fp64 on two (b, h) problems.

    python tools/dq_ab.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import ops


def timeit(fn, iters=3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    torch.manual_seed(0)
    BH, n = 192, 4096
    ds = torch.randn(BH, n, n, device="cuda") * 1e-3
    k = torch.randn(BH, n, 64, device="cuda") * 0.4
    kt = ops.transpose64(k)
    ldt = kt.shape[-1]
    dq32, dq3 = (torch.empty(BH, n, 64, device="cuda") for _ in range(2))

    def f32():
        ops.gemm(a=ds, w=kt, c=dq32, M=n, N=64, K=n, compute=torch.float32, lda=n, sa=(n * n, 0), nb=(BH, 1),
                 ldw=ldt, sw=(64 * ldt, 0), ldc=64, sc=(n * 64, 0))

    planes = ops.split3_rows(kt.view(BH * 64, ldt))

    def s3():
        ops.gemm_n64_split3(ds, planes, dq3, BH, n, n, ldt)

    def split():
        ops.transpose64_split3(k)

    f32(), s3(), split()
    torch.cuda.synchronize()
    ts = {"f32": [], "s3": [], "split": []}
    for _ in range(7):
        ts["f32"].append(timeit(f32))
        ts["s3"].append(timeit(s3))
        ts["split"].append(timeit(split))
    med = {k2: sorted(v)[len(v) // 2] for k2, v in ts.items()}
    ref = ds[:2].double() @ k[:2].double()
    rel = lambda a: ((a[:2].double() - ref).abs().max() / ref.abs().max()).item()  # noqa: E731
    gb = BH * n * n * 4 / 1e9
    flop = 2.0 * BH * n * n * 64
    print(f"dQ BH {BH} Nc = Ns = {n}: dS {gb:.1f} GB", flush=True)
    print(f"  fp32 gemm_n64   {med['f32']:.3f} ms  {gb / med['f32']:.2f} TB/s  {flop / med['f32'] / 1e9:.1f} TF  "
          f"err {rel(dq32):.2e}  (rounds {['%.3f' % t for t in ts['f32']]})")
    print(f"  SPLIT3          {med['s3']:.3f} ms  {gb / med['s3']:.2f} TB/s  {flop / med['s3'] / 1e9:.1f} TF-fp32eq  "
          f"err {rel(dq3):.2e}  (rounds {['%.3f' % t for t in ts['s3']]})")
    print(f"  K^T plane split {med['split'] * 1e3:.1f} us")


if __name__ == "__main__":
    main()
