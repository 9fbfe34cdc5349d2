"""The training step's relu3_1 AdaAttnForLoss kernel alone (mhada_loss_attn: B 8, Nq = Ns = 16384,
d_qk 448, d_v 256, softmax), a few launches with their HIP-event time and TF/s (a target for PMC
passes).   python tools/lossattn_only.py [iters]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import _lib, ops

it = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B, N, Dqk, Dv = 8, 16384, 448, 256
g = torch.Generator(device="cuda").manual_seed(0)
qn = torch.randn(B, N, Dqk, device="cuda", generator=g) * 0.05
kn = torch.randn(B, N, Dqk, device="cuda", generator=g) * 0.05
v = torch.rand(B, N, Dv, device="cuda", generator=g)
x = torch.rand(B, N, Dv, device="cuda", generator=g)
mu = x.mean(dim=1).contiguous()
rs = (1.0 / (x.var(dim=1) + 1e-5).sqrt()).contiguous()
ops.loss_attn(qn, kn, v, x, mu, rs, _lib.ACT_SOFTMAX)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(it):
    ops.loss_attn(qn, kn, v, x, mu, rs, _lib.ACT_SOFTMAX)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / it
flop = 2.0 * B * N * N * (Dqk + 2 * Dv)
print(f"loss_attn relu3_1: {ms:.3f} ms  {flop / ms / 1e9:.1f} TF/s  ({flop / ms / 1e9 / 157.3:.3f} of the fp32 peak)")
