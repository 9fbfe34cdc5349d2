"""In-kernel clock of the bf16 MHAda attention variants (MI355X_MICROARCH.md, DVFS give-back item 6).

Loads the diagnostic build (`make -C mhada-style-transfer_amd/csrc clock` ->
mhada-style-transfer_amd/diag/libmhada_clock.so: the attention kernels stamp the shader clock and
the 100 MHz real-time counter around the key loop into a buffer of their own), runs each variant
back to back for >= 2 s on random data at 1024^2 B4, then reads the last launch's stamps:
clock = d(shader clock) / d(real time) x 100 MHz, median over workgroups.  Also prints the wall
time per launch (HIP events) and the loop's share of the workgroup lifetime.

    python tools/attn_clock.py [variant ...]        (default: fsg fsq1 fsp; "f32": the fp32 kernel at 512^2 B8)
"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import numpy as np
import torch

from mhada_hip import _lib, ops

VARIANTS = {"fsq1": {"attn_fixed_shift": 1}}


def train_dkv(lib):
    """The training dK/dV' kernel at the 512^2 B8 step's shape (the three AdaFormer calls batched:
    BH = 192, Nc = Ns = 4096), with its dS spill."""
    lib.mhada_dbg_train_clock.argtypes = [ctypes.c_void_p, ctypes.c_int]
    torch.manual_seed(0)
    BH, n = 192, 4096
    q, k, v, x = (torch.randn(BH, n, 64, device="cuda") * 0.4 for _ in range(4))
    v = (v - v.mean(dim=1, keepdim=True)).contiguous()
    out, mo, lse = ops.attn_train_fwd(q, k, v, x)
    dmo = torch.randn(BH, n, 128, device="cuda")
    dd = (dmo * mo).sum(-1).contiguous()
    ds = torch.empty(BH, n, n, device="cuda")
    dk, dv = torch.empty_like(k), torch.empty_like(v)
    st = torch.cuda.current_stream().cuda_stream
    run = lambda: lib.mhada_attn_train_dkv(q.data_ptr(), k.data_ptr(), v.data_ptr(), lse.data_ptr(),  # noqa: E731
                                           dmo.data_ptr(), dd.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                                           ds.data_ptr(), BH, n, n, st)
    flop = 768.0 * BH * n * n
    nblk = BH * (n // 128)
    for rnd in range(2):
        t0, cnt = time.time(), 0
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        while time.time() - t0 < 2.0:
            run()
            cnt += 1
            torch.cuda.synchronize()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / cnt
        buf = np.zeros(4 * nblk, dtype=np.uint64)
        assert lib.mhada_dbg_train_clock(buf.ctypes.data, 4 * nblk) == 0, lib.mhada_last_error()
        st4 = buf.reshape(nblk, 4).astype(np.float64)
        dclk, drt = st4[:, 2] - st4[:, 0], st4[:, 3] - st4[:, 1]
        ok = drt > 0
        ghz = np.median(dclk[ok] / drt[ok]) * 0.1
        print(f"round {rnd} dkv   {ms:.3f} ms/launch  {flop / ms / 1e9:7.1f} TF/s  in-kernel clock {ghz:.3f} GHz "
              f"(median of {ok.sum()} workgroups)  {flop / ms / 1e9 / (ghz * 1024 * 64 * 1e-3):.3f} of the "
              f"clock-adjusted fp32 peak ({flop / ms / 1e9 / 157.3:.3f} of the nominal)", flush=True)


def main():
    lib = _lib.load(os.path.join(REPO, "mhada-style-transfer_amd", "diag", "libmhada_clock.so"))
    _lib._lib = lib
    lib.mhada_dbg_attn_clock.argtypes = [ctypes.c_void_p, ctypes.c_int]
    names = sys.argv[1:] or ["fsg", "fsq1", "fsp"]
    if names == ["dkv"]:
        return train_dkv(lib)
    torch.manual_seed(0)
    f32 = names == ["f32"]  # the fp32 kernel at 512^2 B8 (the headline's attention)
    B, H, nc, ns = (8, 8, 4096, 4096) if f32 else (4, 8, 16384, 16384)
    dt = torch.float32 if f32 else torch.bfloat16
    q = (torch.randn(B, H, nc, 64, device="cuda") * 0.35).to(dt)
    kv = (torch.randn(B, H, ns, 128, device="cuda") * 0.35).to(dt)
    vt = ops.transpose_v(kv)
    fcs = torch.randn(B, nc, 512, device="cuda")
    mu, rs = ops.instnorm_stats(fcs)
    vmu = torch.zeros(B, 512, device="cuda")
    nblk = B * H * (nc // 256)
    flop = 6.0 * nc * ns * 512 * B
    for rnd in range(2):
        for v in names:
            with _lib.tuning(**VARIANTS.get(v, {})):
                run = lambda: ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)  # noqa: E731
                t0 = time.time()
                n = 0
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                while time.time() - t0 < 2.0:
                    for _ in range(5):
                        run()
                    n += 5
                    torch.cuda.synchronize()
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / n
                run()
                torch.cuda.synchronize()
            # the persistent kernel stamps per workgroup (its last block): one entry per CU
            nst = min(nblk, torch.cuda.get_device_properties(0).multi_processor_count) if v == "fsp" else nblk
            buf = np.zeros(4 * nst, dtype=np.uint64)
            assert lib.mhada_dbg_attn_clock(buf.ctypes.data, 4 * nst) == 0, lib.mhada_last_error()
            st = buf.reshape(nst, 4).astype(np.float64)
            dclk, drt = st[:, 2] - st[:, 0], st[:, 3] - st[:, 1]
            ok = drt > 0
            ghz = np.median(dclk[ok] / drt[ok]) * 0.1
            loop_us = np.median(drt[ok]) / 100.0
            print(f"round {rnd} {v:5s} {ms:.3f} ms/launch  {flop / ms / 1e9:7.1f} TF/s  in-kernel clock "
                  f"{ghz:.3f} GHz (median of {ok.sum()} workgroups; p10 {np.percentile(dclk[ok] / drt[ok], 10) * 0.1:.3f},"
                  f" p90 {np.percentile(dclk[ok] / drt[ok], 90) * 0.1:.3f})  loop {loop_us:.1f} us/workgroup  "
                  f"{flop / ms / 1e9 / (ghz * 1024 * (64 if f32 else 1024) * 1e-3):.3f} of the clock-adjusted "
                  f"{'fp32' if f32 else 'bf16'} peak", flush=True)


if __name__ == "__main__":
    main()
