"""Errors of the SPLIT3 attention against fp64 on tests/test_gpu_kernels.py's late-max-jump cases
(the fixed shift's exact recompute path) beside the fp32-MFMA kernel's, per case and wave count.

    python tools/s3_late_jump_err.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd"), os.path.join(REPO, "tests")]

from mhada_hip import _lib, ops  # noqa: E402
from test_gpu_kernels import S3_WAVES, _attn_ref, rel, rnd  # noqa: E402


def main():
    for kernel in S3_WAVES:
        for Nc, Ns in [(300, 700), (256, 128), (97, 33), (256, 1024), (97, 384)]:
            B, H = 1, 8
            q = rnd(B, H, Nc, 64, seed=11)
            q = q / q.norm(dim=-1, keepdim=True) * 4.0
            kv = rnd(B, H, Ns, 128, scale=0.1, seed=12)
            late = Ns - 5
            kv[:, :, late, :64] = 30.0 * q[:, :, : min(Nc, 1), :].mean(dim=2)
            kv[:, :, late - 1, :64] = -kv[:, :, late, :64]
            vt = ops.transpose_v(kv)
            fcs = rnd(B, Nc, 512, seed=13)
            mu, rs = ops.instnorm_stats(fcs)
            vmu = rnd(B, 512, seed=14)
            img = ops.split3_kv(kv, vt)
            with _lib.tuning(**S3_WAVES[kernel]):
                y = ops.attn_split3(q, img, Ns, fcs, mu, rs, vmu)
            y32 = ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
            ref = _attn_ref(q, kv, fcs, mu, rs, vmu)
            e3, e32 = rel(y, ref), rel(y32, ref)
            print(f"{kernel} Nc {Nc:4d} Ns {Ns:5d}: split3 {e3:.2e}  fp32 {e32:.2e}  ratio {e3 / e32:.2f}", flush=True)


if __name__ == "__main__":
    main()
