"""The MHAda K|V' projection (N = 128 with the V'^T | V'^2^T image epilogue) alone, for rocprofv3
PMC passes: python tools/proj_only.py [bf16|f32] [B] [N] [iters]   (default bf16 4 16384 20, the
configs[2] shape; A = fp32 fs rows [B][N][512], 8 heads of 64)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch

from mhada_hip import ops


def main():
    dt = torch.float32 if (len(sys.argv) > 1 and sys.argv[1] == "f32") else torch.bfloat16
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    H, C, dev = 8, 512, "cuda"
    torch.manual_seed(0)
    x = torch.randn(B, N, C, device=dev)
    mu = x.mean(dim=1)
    wkv = (torch.randn(B, H, 128, 64, device=dev) / 8).to(dt)
    bkv = torch.randn(H, 128, device=dev)
    kv = torch.empty(B, H, N, 128, device=dev, dtype=dt)
    ldt = (N + 63) // 64 * 64
    vt = torch.empty(B, H, 128, ldt, device=dev, dtype=dt)
    ka = dict(a=x, w=wkv, c=kv, M=N, N=128, K=64, compute=dt, lda=C, sa=(N * C, 64), nb=(B, H), a_mu=mu,
              smu=(C, 64), ldw=64, sw=(H * 8192, 8192), bias=bkv, sb=(0, 128), ldc=128,
              sc=(H * N * 128, N * 128), vt=vt, ldt=ldt, svt=(H * 128 * ldt, 128 * ldt))
    if os.environ.get("PROJ_AB"):  # A/B of a tuning knob: same vt / K bits, interleaved timing
        from mhada_hip import _lib
        knob, val = os.environ["PROJ_AB"].split("=")
        ops.gemm(**ka)
        ref_vt, ref_k = vt.clone(), kv[..., :64].clone()
        vt.fill_(float("nan"))
        with _lib.tuning(**{knob: int(val)}):
            ops.gemm(**ka)
        torch.cuda.synchronize()
        assert torch.equal(vt, ref_vt) and torch.equal(kv[..., :64], ref_k), "A/B outputs differ"
        ts = {"base": [], knob + "=" + val: []}
        for _ in range(7):
            for k in ts:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with _lib.tuning(**({} if k == "base" else {knob: int(val)})):
                    s.record()
                    for _ in range(10):
                        ops.gemm(**ka)
                    e.record()
                torch.cuda.synchronize()
                ts[k].append(s.elapsed_time(e) / 10 * 1e3)
        print(" ".join(f"{k} {sorted(v)[3]:.1f} us" for k, v in ts.items()), "(bit-identical)")
    for _ in range(iters):
        ops.gemm(**ka)
    torch.cuda.synchronize()
    es = x.element_size() * B * N * C + kv.element_size() * B * H * N * (64 + 2 * 64)
    print(f"proj {str(dt)[6:]} B{B} N{N}: algorithmic bytes per launch {es / 1e6:.1f} MB "
          f"(A fp32 read, K half + V'^T|V'^2^T written)")


if __name__ == "__main__":
    main()
