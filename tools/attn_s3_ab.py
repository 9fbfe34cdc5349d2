"""A/B of the fp32 MHAda attention: the fp32-MFMA kernel (attn_f32_kernel, mhada_attn) against the
SPLIT3 kernel on the bf16 MFMA (attn_s3_kernel, mhada_attn_split3; round 6), in one process,
interleaved rounds, median of rounds, at the bench shapes.  Also the one-time plane split
(mhada_split3_kv) and each kernel's error against fp64 on a row subset.

    python tools/attn_s3_ab.py [waves...]      (waves: 0 = auto, 4, 8)
    S3_VARIANTS="base: inter:xknob=1 noprio:attn_prio=0" python tools/attn_s3_ab.py   (tuning A/B)
"""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch

from mhada_hip import _lib, ops

if os.environ.get("S3_LIB"):  # an alternative build of the library (A/B of compile options)
    _lib.LIB_PATH = os.path.abspath(os.environ["S3_LIB"])

SHAPES = [("512^2 B8", 8, 4096, 4096), ("512^2 B1", 1, 4096, 4096), ("video 1080p/s256", 1, 32400, 1024),
          ("1024^2 B4", 4, 16384, 16384), ("ragged", 2, 1000, 777)]


def timeit(fn, rounds=7, iters=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters)
    return sorted(ts)[len(ts) // 2]


def ref_rows(q, kv, fcs, mu, rs, vmu, rows):
    """fp64 mhada_attn for query rows `rows` of every (b, h)."""
    B, H, Nc, _ = q.shape
    qd, kd, vd = q[:, :, rows].double(), kv[..., :64].double(), kv[..., 64:].double()
    a = torch.softmax(qd @ kd.transpose(-1, -2) * math.log(2.0), dim=-1)
    m = a @ vd
    e2 = a @ (vd * vd)
    s = torch.sqrt(torch.clamp(e2 - m * m, min=1e-6))
    out = s.permute(0, 2, 1, 3).reshape(B, len(rows), H * 64)
    mm = m.permute(0, 2, 1, 3).reshape(B, len(rows), H * 64)
    f = (fcs[:, rows].double() - mu.double()[:, None]) * rs.double()[:, None]
    return out * f + mm + vmu.double()[:, None]


def main():
    waves = [int(x) for x in sys.argv[1:]] or [0]
    variants = []
    for item in os.environ.get("S3_VARIANTS", "base:").split():
        name, _, kv = item.partition(":")
        variants.append((name, {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}))
    torch.manual_seed(0)
    H = 8
    for name, B, nc, ns in SHAPES:
        q = torch.randn(B, H, nc, 64, device="cuda") * 0.5
        kv = torch.randn(B, H, ns, 128, device="cuda") * 0.5
        vt = ops.transpose_v(kv)
        fcs = torch.randn(B, nc, 512, device="cuda")
        mu, rs = ops.instnorm_stats(fcs)
        vmu = torch.zeros(B, 512, device="cuda")
        img = ops.split3_kv(kv, vt)
        rows = torch.arange(0, nc, max(1, nc // 256), device="cuda")
        ref = ref_rows(q, kv, fcs, mu, rs, vmu, rows)
        fl = 6.0 * nc * ns * 512 * B
        y32 = ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
        e32 = ((y32[:, rows].double() - ref).norm() / ref.norm()).item()
        t32 = timeit(lambda: ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0))
        tsp = timeit(lambda: ops.split3_kv(kv, vt))
        line = f"{name:18s} f32 {t32:.3f} ms {fl / t32 / 1e9:.1f} TF (err {e32:.2e}) | split3_kv {tsp * 1e3:.1f} us"
        for w in waves:
            for vname, knobs in variants:
                with _lib.tuning(attn_waves=w, **knobs):
                    y = ops.attn_split3(q, img, ns, fcs, mu, rs, vmu)
                    es = ((y[:, rows].double() - ref).norm() / ref.norm()).item()
                    ts = timeit(lambda: ops.attn_split3(q, img, ns, fcs, mu, rs, vmu))
                # bf16 MFMA FLOP per (query, key, head): 6 x 128 (QK) + 6 x 256 (PV) + 3 x 32 (row sum)
                mf = fl / 384 * (6 * 128 + 6 * 256 + 96) / 1e9  # GFLOP
                line += (f" | s3 {vname} w{w} {ts:.3f} ms {fl / ts / 1e9:.1f} TF-fp32eq, bf16 pipe {mf / ts:.0f} TF ="
                         f" {mf / ts / 2500:.3f} (err {es:.2e}) x{t32 / ts:.2f}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
