"""A/B of two builds of libmhada_hip.so in ONE process (cdna_hip_programming.md rule 24):
interleaved rounds of the bf16 / fp32 attention and the bench GEMM shapes, median per build.

    python tools/lib_ab.py <libA.so> <libB.so>
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch

from mhada_hip import _lib, ops

LIBS = {"A": _lib.load(sys.argv[1]), "B": _lib.load(sys.argv[2])}


def use(name):
    _lib._lib = LIBS[name]


def timed(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def ab(label, fn, flop, rounds=9):
    t = {"A": [], "B": []}
    for k in t:
        use(k)
        fn()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k in t:
            use(k)
            t[k].append(timed(fn))
    med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
    print(f"{label:40s} A {med['A'] * 1e3:8.1f} us {flop / med['A'] / 1e9:7.1f} TF   "
          f"B {med['B'] * 1e3:8.1f} us {flop / med['B'] / 1e9:7.1f} TF   B/A time {med['B'] / med['A']:.3f}", flush=True)


def main():
    torch.manual_seed(0)
    H = 8
    for name, B, nc, ns, dt in (("attn bf16 1024^2 B4", 4, 16384, 16384, torch.bfloat16),
                                ("attn f32 512^2 B8", 8, 4096, 4096, torch.float32),
                                ("attn bf16 video", 1, 32400, 1024, torch.bfloat16)):
        q = (torch.randn(B, H, nc, 64, device="cuda") * 0.35).to(dt)
        kv = (torch.randn(B, H, ns, 128, device="cuda") * 0.35).to(dt)
        vt = ops.transpose_v(kv)
        fcs = torch.randn(B, nc, 512, device="cuda")
        mu, rs = ops.instnorm_stats(fcs)
        vmu = torch.zeros(B, 512, device="cuda")
        ab(name, lambda: ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0), 6.0 * nc * ns * 512 * B)
    for (M, N, K, res) in ((65536, 1536, 512, False), (65536, 2048, 512, False), (65536, 512, 2048, True),
                           (65536, 512, 512, True)):
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        b = torch.randn(N, device="cuda")
        r = torch.randn(M, N, device="cuda") if res else None
        out = torch.float32 if res else torch.bfloat16
        ab(f"gemm bf16 {M}x{N}x{K} res={int(res)}", lambda: ops.linear(x, w, b, out, residual=r), 2.0 * M * N * K)


if __name__ == "__main__":
    main()
