"""HIP-event time of mhada_loss_attn at the train step's relu3_1 / relu4_1 / relu5_1 shapes
(512^2 batch 8).  usage: python tools/loss_attn_time.py"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import ops
from mhada_hip._lib import ACT_SOFTMAX

for (N, dqk, dv) in [(16384, 448, 256), (4096, 960, 512), (1024, 1472, 512)]:
    B = 8
    q = torch.randn(B, N, dqk, device="cuda") * 0.05
    k = torch.randn(B, N, dqk, device="cuda") * 0.05
    v = torch.rand(B, N, dv, device="cuda")
    x = torch.rand(B, N, dv, device="cuda")
    mu, rs = x.mean(1), 1 / x.std(1)
    f = lambda: ops.loss_attn(q, k, v, x, mu, rs, ACT_SOFTMAX)  # noqa: E731
    flop = B * N * N * (2 * dqk + 4 * dv)
    f(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        f()
    e.record(); torch.cuda.synchronize()
    t = s.elapsed_time(e) / 3
    print(f"N={N} dqk={dqk} dv={dv}: {t:.2f} ms  {flop / t / 1e9:.1f} TF/s", flush=True)
