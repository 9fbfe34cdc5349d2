"""Per-op microbenchmarks on the GPU (interleaved rounds in one process, median of rounds).

    python tools/opbench.py [gemm|conv|attn|cosine|all]     (attn: tools/attn_ab.py)

GEMM shapes are the forward path's (1024^2 batch 4 -> M = 65536 tokens); hipBLASLt via
torch.matmul is timed beside ours on the same operands as a calibration point.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch

from mhada_hip import ops


def bench(fns, rounds=7, iters=10):
    """fns: {name: callable}; returns {name: median ms per call}."""
    times = {k: [] for k in fns}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                f()
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / iters)
    return {k: sorted(v)[len(v) // 2] for k, v in times.items()}


def with_env(key, val, fn, *a, **k):
    """Run fn with one kernel-variant knob changed (MHADA_<KNOB> naming, see include/mhada_hip.h)."""
    from mhada_hip import _lib
    with _lib.tuning(**{key[len("MHADA_"):].lower(): int(val)}):
        return fn(*a, **k)


def gemm_suite(dts=(torch.bfloat16, torch.float32)):
    dev = "cuda"
    for dt in dts:
        M = 65536 if dt == torch.bfloat16 else 32768
        for (N, K, out, res, relu) in [(1536, 512, dt, False, False), (2048, 512, dt, False, True),
                                       (512, 2048, torch.float32, True, False), (512, 512, torch.float32, True, False)]:
            x = torch.randn(M, K, device=dev).to(dt)
            w = (torch.randn(N, K, device=dev) / K ** 0.5).to(dt)
            b = torch.randn(N, device=dev)
            r = torch.randn(M, N, device=dev) if res else None
            fns = {"ours": lambda: ops.linear(x, w, b, out, residual=r, relu=relu),
                   "torch": lambda: torch.addmm(b.to(dt), x, w.t())}
            fns["epi_direct"] = lambda: with_env("MHADA_GEMM_LDSEPI", "0", ops.linear, x, w, b, out, residual=r,
                                                 relu=relu)
            if res:
                fns["no_rinit"] = lambda: with_env("MHADA_GEMM_RINIT", "0", ops.linear, x, w, b, out, residual=r,
                                                   relu=relu)
            if dt == torch.bfloat16:
                fns["oneshot"] = lambda: with_env("MHADA_GEMM_PERSIST", "0", ops.linear, x, w, b, out, residual=r,
                                                  relu=relu)
            else:
                fns["tile128"] = lambda: with_env("MHADA_GEMM_PP", "0", ops.linear, x, w, b, out, residual=r,
                                                  relu=relu)

            t = bench(fns)
            fl = 2 * M * N * K
            print(f"gemm {str(dt)[6:]:8s} M={M} N={N:5d} K={K:5d} out={str(out)[6:]:8s} res={res:d}: "
                  + "  ".join(f"{k} {v * 1e3:7.1f} us {fl / v / 1e9:7.1f} TF" for k, v in t.items()))


def gemm_k_suite():
    """Main-loop rate vs K: the same M x N at growing K separates the per-tile prologue/epilogue
    cost (fixed per tile) from the K-loop rate."""
    dev = "cuda"
    M, N = 65536, 1536
    for K in (512, 1024, 2048, 4096):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        t = bench({"ours": lambda: ops.linear(x, w, b, torch.bfloat16),
                   "epi_direct": lambda: with_env("MHADA_GEMM_LDSEPI", "0", ops.linear, x, w, b, torch.bfloat16),
                   "torch": lambda: torch.addmm(b.to(torch.bfloat16), x, w.t())})
        fl = 2 * M * N * K
        print(f"gemmK bf16 M={M} N={N} K={K:5d}: " + "  ".join(f"{k} {v * 1e3:7.1f} us {fl / v / 1e9:7.1f} TF"
                                                             for k, v in t.items()))
    # the fp32-out residual form (ViT out_proj / MLP2, MHAda out_conv): HBM rate vs K, with and
    # without the residual, so the fixed per-tile R-load / C-store cost separates from the K loop
    N = 512
    for K in (512, 1024, 2048):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev)
        t = bench({"res": lambda: ops.linear(x, w, b, torch.float32, residual=r),
                   "nores": lambda: ops.linear(x, w, b, torch.float32),
                   "bf16out": lambda: ops.linear(x, w, b, torch.bfloat16),
                   "no_rinit": lambda: with_env("MHADA_GEMM_RINIT", "0", ops.linear, x, w, b, torch.float32, residual=r)})
        by = {"res": M * K * 2 + 2 * M * N * 4, "nores": M * K * 2 + M * N * 4, "bf16out": M * K * 2 + M * N * 2,
              "no_rinit": M * K * 2 + 2 * M * N * 4}
        print(f"gemmR bf16 M={M} N={N} K={K:5d}: " + "  ".join(f"{k} {v * 1e3:7.1f} us {by[k] / v / 1e6:7.1f} GB/s"
                                                             for k, v in t.items()))


def gemm_k32_suite():
    """fp32 main-loop rate vs K for the ping-pong and the one-wave-per-SIMD kernels: the slope
    separates the K-loop rate from the fixed per-tile prologue / epilogue cost."""
    dev = "cuda"
    M = 32768
    for N in (512, 1536):
        for K in (512, 1024, 2048, 4096):
            x = torch.randn(M, K, device=dev)
            w = torch.randn(N, K, device=dev) / K ** 0.5
            b = torch.randn(N, device=dev)
            t = bench({"pp": lambda: ops.linear(x, w, b, torch.float32),
                       "torch": lambda: torch.addmm(b, x, w.t())})
            fl = 2 * M * N * K
            print(f"gemmK f32 M={M} N={N:5d} K={K:5d}: " + "  ".join(f"{k} {v * 1e3:7.1f} us {fl / v / 1e9:7.1f} TF"
                                                                  for k, v in t.items()))


def out3_suite():
    dev = "cuda"
    for dt, B, res in ((torch.bfloat16, 4, 1024), (torch.float32, 8, 512)):
        x = torch.rand(B, res, res, 64, device=dev).to(dt)
        w = torch.randn(3, 3, 64, 3, device=dev) * 0.05
        b = torch.randn(3, device=dev)
        fns = {"default": lambda: ops.conv3x3_out3(x, w, b)}
        if dt == torch.bfloat16:
            fns["valu"] = lambda: with_env("MHADA_OUT3_MFMA", "0", ops.conv3x3_out3, x, w, b)
        else:
            fns["per_pixel"] = lambda: with_env("MHADA_OUT3_TILE", "0", ops.conv3x3_out3, x, w, b)
        t = bench(fns)
        by = x.numel() * x.element_size() + B * 3 * res * res * 4
        print(f"out3 {str(dt)[6:]:8s} B={B} {res}^2: " + "  ".join(f"{k} {v * 1e3:8.1f} us {by / v / 1e6:7.1f} GB/s"
                                                                for k, v in t.items()))


def conv_suite():
    dev = "cuda"
    for dt, B, res in ((torch.bfloat16, 4, 1024), (torch.float32, 8, 512)):
        h = res // 8
        for (Ci, Co, H, up) in [(512, 256, h, False), (256, 256, 2 * h, True), (256, 256, 2 * h, False),
                                (256, 128, 2 * h, False), (128, 128, 4 * h, True), (128, 64, 4 * h, False),
                                (64, 64, 8 * h, True)]:
            Hin = H // 2 if up else H
            x = torch.rand(B, Hin, Hin, Ci, device=dev).to(dt)
            w = (torch.randn(Co, 9 * Ci, device=dev) / (9 * Ci) ** 0.5).to(dt)
            bias = torch.randn(Co, device=dev)
            fns = {"fused": lambda: ops.conv3x3(x, w, bias, dt, upsample=up)}
            if not up:  # MIOpen calibration point (zero padding, channels-last, same shape)
                xc = x.permute(0, 3, 1, 2)
                w4 = w.view(Co, 3, 3, Ci).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
                fns["miopen"] = lambda: torch.nn.functional.conv2d(xc, w4, bias.to(dt), padding=1)
            if dt == torch.float32 and Co > 128:
                fns["tile128"] = lambda: with_env("MHADA_GEMM_PP", "0", ops.conv3x3, ops.upsample2x(x) if up else x, w,
                                                  bias, dt, upsample=False)
            if dt == torch.bfloat16 and 64 < Co <= 128:
                fns["pp128_off"] = lambda: with_env("MHADA_GEMM_PP128", "0", ops.conv3x3, ops.upsample2x(x) if up else x,
                                                    w, bias, dt, upsample=False)
            if Co > 128 and not (dt == torch.float32 and up):
                fns["epi_direct"] = lambda: with_env("MHADA_GEMM_LDSEPI", "0", ops.conv3x3, x, w, bias, dt, upsample=up)
            if dt == torch.bfloat16 and not up and Co > 128:
                fns["oneshot"] = lambda: with_env("MHADA_GEMM_PERSIST", "0", ops.conv3x3, x, w, bias, dt,
                                                  upsample=False)
            if dt == torch.bfloat16 and (Ci, Co) in ((128, 64), (128, 128), (256, 128)) and not up:
                fns["dir_off"] = lambda: with_env("MHADA_CONV_DIR", "0", ops.conv3x3, x, w, bias, dt, upsample=False)
            if Co <= 64:
                fns["n64_256"] = lambda: with_env("MHADA_GEMM_N64", "256", ops.conv3x3, ops.upsample2x(x) if up else x, w,
                                                  bias, dt, upsample=False)
            if up:
                fns["sep"] = lambda: ops.conv3x3(ops.upsample2x(x), w, bias, dt, upsample=False)
                fns["upsample_only"] = lambda: ops.upsample2x(x)
                fns["upsample_pp"] = lambda: with_env("MHADA_XKNOB", "1", ops.upsample2x, x)
            t = bench(fns)
            fl = 2 * B * H * H * Co * 9 * Ci
            print(f"conv {str(dt)[6:]:8s} {Ci:3d}->{Co:3d} @{H:4d} up={up:d}: "
                  + "  ".join(f"{k} {v * 1e3:8.1f} us {fl / v / 1e9:7.1f} TF" for k, v in t.items()))


def n64_suite():
    """fp32 N = 64 GEMMs of the training step: the attention backward's dQ = dS K (24 images x 8
    heads at 64^2 tokens) and the grouped per-head 1x1 convs (K = 64): the LDS-DMA ring kernel vs
    torch.bmm."""
    dev = "cuda"
    for nz, M, K, lda in ((192, 4096, 4096, 4096), (8, 98304, 64, 512), (8, 98304, 64, 64)):
        a = torch.randn(nz, M, lda, device=dev) if lda == K else torch.randn(M, lda, device=dev)
        w = torch.randn(nz, 64, K, device=dev) / K ** 0.5
        c = torch.empty(nz, M, 64, device=dev)
        sa = (M * K, 0) if lda == K else (64, 0)
        args = dict(a=a, w=w, c=c, M=M, N=64, K=K, compute=torch.float32, lda=lda, sa=sa, nb=(nz, 1), ldw=K,
                    sw=(64 * K, 0), ldc=64, sc=(M * 64, 0))
        fns = {"default": lambda: ops.gemm(**args)}
        if lda == K:
            fns["torch"] = lambda: torch.bmm(a, w.transpose(1, 2))
        t = bench(fns, rounds=5, iters=3)
        fl = 2 * nz * M * 64 * K
        by = 4 * nz * M * (K + 64)
        print(f"n64 fp32 z={nz} M={M} K={K}: " + "  ".join(f"{k} {v * 1e3:8.1f} us {fl / v / 1e9:6.1f} TF "
                                                        f"{by / v / 1e6:6.0f} GB/s" for k, v in t.items()))
        del a


def proj_suite():
    """The MHAda block's per-head projections as engine.block_forward issues them (512^2 B8:
    Nc = Ns = 4096, 8 heads, fp32 and bf16): q (N = 64, centred A) and K|V' (N = 128 with the
    V'^T image); plus the uncentred q form (which routes to the fp32 LDS-DMA ring kernel)."""
    dev = "cuda"
    H, C = 8, 512
    for B, N, dt in ((8, 4096, torch.float32), (8, 4096, torch.bfloat16), (4, 16384, torch.bfloat16)):
        x = torch.randn(B, N, C, device=dev)
        mu = x.mean(dim=1)
        wq = (torch.randn(B, H, 64, 64, device=dev) / 8).to(dt)
        wkv = (torch.randn(B, H, 128, 64, device=dev) / 8).to(dt)
        bq = torch.randn(H, 64, device=dev)
        bkv = torch.randn(H, 128, device=dev)
        q = torch.empty(B, H, N, 64, device=dev, dtype=dt)
        kv = torch.empty(B, H, N, 128, device=dev, dtype=dt)
        vt = torch.empty(B, H, 128, N, device=dev, dtype=dt)
        qa = dict(a=x, w=wq, c=q, M=N, N=64, K=64, compute=dt, lda=C, sa=(N * C, 64), nb=(B, H), ldw=64,
                  sw=(H * 4096, 4096), bias=bq, sb=(0, 64), ldc=64, sc=(H * N * 64, N * 64))
        ka = dict(a=x, w=wkv, c=kv, M=N, N=128, K=64, compute=dt, lda=C, sa=(N * C, 64), nb=(B, H), a_mu=mu,
                  smu=(C, 64), ldw=64, sw=(H * 8192, 8192), bias=bkv, sb=(0, 128), ldc=128,
                  sc=(H * N * 128, N * 128), vt=vt, ldt=N, svt=(H * 128 * N, 128 * N))
        fns = {"q": lambda: ops.gemm(a_mu=mu, smu=(C, 64), **qa),
               "q_n64_256": lambda: with_env("MHADA_GEMM_N64", "256", ops.gemm, a_mu=mu, smu=(C, 64), **qa),
               "q_uncentred": lambda: ops.gemm(**qa),
               "kv_vt": lambda: ops.gemm(**ka)}
        t = bench(fns)
        qb, kb = 4 * B * N * C // 8 + B * H * N * 64 * q.element_size(), 4 * B * N * C // 8 + 3 * B * H * N * 64 * q.element_size()
        print(f"proj {str(dt)[6:]:8s} B{B} N{N}: " + "  ".join(
            f"{k} {v * 1e3:6.1f} us {(kb if k.startswith('kv') else qb) / v / 1e6:6.0f} GB/s" for k, v in t.items()))


def cosine_suite():
    """The cosine activation: the flash loop (mhada_attn ACT_COSINE) vs the linear form
    (mhada_cosine_moments once per style + mhada_cosine_attn per call) at the bench shapes."""
    from mhada_hip import _lib
    dev = "cuda"
    for B, N, dt in ((8, 4096, torch.float32), (4, 16384, torch.bfloat16)):
        H, C = 8, 512
        q = torch.randn(B, H, N, 64, device=dev).to(dt)
        kv = torch.randn(B, H, N, 128, device=dev).to(dt)
        vt = ops.transpose_v(kv)
        ops.cosine_prep(q, kv)
        fcs = torch.randn(B, N, C, device=dev)
        mu, rs, vmu = torch.zeros(B, C, device=dev), torch.ones(B, C, device=dev), torch.zeros(B, C, device=dev)
        mom = ops.cosine_moments(kv, vt)
        fns = {"flash": lambda: ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, _lib.ACT_COSINE),
               "moments": lambda: ops.cosine_moments(kv, vt),
               "apply": lambda: ops.cosine_attn(q, mom, fcs, mu, rs, vmu)}
        t = bench(fns, rounds=5, iters=3)
        print(f"cosine {str(dt)[6:]:8s} B{B} N{N}: " + "  ".join(f"{k} {v * 1e3:8.1f} us" for k, v in t.items()))


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    torch.manual_seed(0)
    if what in ("gemm", "all"):
        gemm_suite()
    if what == "gemm32":
        gemm_suite((torch.float32,))
    if what in ("gemmk",):
        gemm_k_suite()
    if what == "gemmk32":
        gemm_k32_suite()
    if what in ("n64",):
        n64_suite()
    if what == "proj":
        proj_suite()
    if what == "cosine":
        cosine_suite()
    if what in ("conv", "all"):
        conv_suite()
    if what in ("out3", "conv", "all"):
        out3_suite()
    if what in ("attn", "all"):
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import attn_ab  # the attention kernel variants (MHADA_ATTN_* switches)
        attn_ab.main()
