"""The bench's GEMM shapes in isolation, in a fixed launch order, as the target of rocprofv3
FETCH_SIZE / WRITE_SIZE passes (tools/gemm_traffic.sh -> tools/gemm_traffic_sum.py): the fp32 ViT's
SPLIT3 GEMMs at 512^2 B8 (QKV, MLP1 -> planes, MLP2 + residual; M = 32768) and the bf16 path's
fp32-out residual GEMMs at 1024^2 B4 (out_proj K = 512 and MLP2 K = 2048, M = 65536).  Each shape runs
REPS times after one warm-up launch; LAUNCHES below is the order the summary script relies on.

    python tools/gemm_traffic_shapes.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import ops

REPS = 3
# (name, algorithmic read bytes, algorithmic write bytes)
LAUNCHES = []


def main():
    torch.manual_seed(0)
    dev = "cuda"
    M, C = 32768, 512
    x = torch.randn(M, C, device=dev)
    planes = ops.split3_rows(x)
    w_qkv = ops.split3_weight(torch.randn(3 * C, C, device=dev) * C ** -0.5)
    w1 = ops.split3_weight(torch.randn(4 * C, C, device=dev) * C ** -0.5)
    w2 = ops.split3_weight(torch.randn(C, 4 * C, device=dev) * (4 * C) ** -0.5)
    b3, b4, b1 = (torch.zeros(n, device=dev) for n in (3 * C, 4 * C, C))
    res = torch.randn(M, C, device=dev)
    m1 = ops.linear_split3(planes, w1, b4, torch.float32, relu=True, out_planes=True)
    shapes = [
        ("split3_qkv_512b8", lambda: ops.linear_split3(planes, w_qkv, b3, torch.float32),
         3 * M * C * 2 + 3 * C * 6 * C * 2, M * 3 * C * 4),
        ("split3_mlp1_planes_512b8", lambda: ops.linear_split3(planes, w1, b4, torch.float32, relu=True, out_planes=True),
         3 * M * C * 2 + 4 * C * 6 * C * 2, 3 * M * 4 * C * 2),
        ("split3_mlp2_res_512b8", lambda: ops.linear_split3(m1, w2, b1, torch.float32, residual=res),
         3 * M * 4 * C * 2 + C * 6 * 4 * C * 2 + M * C * 4, M * C * 4),
    ]
    Mb = 65536
    a512 = torch.randn(Mb, C, device=dev).to(torch.bfloat16)
    a2048 = torch.randn(Mb, 4 * C, device=dev).to(torch.bfloat16)
    wo = (torch.randn(C, C, device=dev) * C ** -0.5).to(torch.bfloat16)
    w2b = (torch.randn(C, 4 * C, device=dev) * (4 * C) ** -0.5).to(torch.bfloat16)
    rb = torch.randn(Mb, C, device=dev)
    shapes += [
        ("bf16_outproj_res_1024b4", lambda: ops.linear(a512, wo, b1, torch.float32, residual=rb),
         Mb * C * 2 + C * C * 2 + Mb * C * 4, Mb * C * 4),
        ("bf16_mlp2_res_1024b4", lambda: ops.linear(a2048, w2b, b1, torch.float32, residual=rb),
         Mb * 4 * C * 2 + C * 4 * C * 2 + Mb * C * 4, Mb * C * 4),
    ]
    for name, fn, rd, wr in shapes:
        fn()  # warm-up launch (its counters are skipped by the summary)
        torch.cuda.synchronize()
        for _ in range(REPS):
            fn()
        torch.cuda.synchronize()
        LAUNCHES.append((name, rd, wr))
    for name, rd, wr in LAUNCHES:
        print(f"shape {name} algorithmic_read {rd} algorithmic_write {wr}", flush=True)


if __name__ == "__main__":
    main()
