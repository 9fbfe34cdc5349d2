"""The training dK/dV' kernel (with the dS spill) alone at the 512^2 B8 step's shape (BH = 192,
Nc = Ns = 4096), a few launches (a target for rocprofv3 PMC passes).
    python tools/dkv_only.py [train_dkv_dma: 0|1]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

from mhada_hip import _lib, ops

if len(sys.argv) > 1:
    _lib.set_tuning("train_dkv_dma", int(sys.argv[1]))
torch.manual_seed(0)
BH, n = 192, 4096
q, k, v, x = (torch.randn(BH, n, 64, device="cuda") * 0.4 for _ in range(4))
v = (v - v.mean(dim=1, keepdim=True)).contiguous()
out, mo, lse = ops.attn_train_fwd(q, k, v, x)
dmo = torch.randn(BH, n, 128, device="cuda")
dd = (dmo * mo).sum(-1).contiguous()
ds = torch.empty(BH, n, n, device="cuda")
dk, dv = torch.empty_like(k), torch.empty_like(v)
lib = _lib.load()


def launch():
    assert lib.mhada_attn_train_dkv(q.data_ptr(), k.data_ptr(), v.data_ptr(), lse.data_ptr(), dmo.data_ptr(),
                                    dd.data_ptr(), dk.data_ptr(), dv.data_ptr(), ds.data_ptr(), BH, n, n,
                                    torch.cuda.current_stream().cuda_stream) == 0


launch()
torch.cuda.synchronize()
iters = int(os.environ.get("ITERS", "3"))
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(iters):
    launch()
e.record()
torch.cuda.synchronize()
t = s.elapsed_time(e) / iters
fl = 2 * BH * n * n * 64 * 6  # S, dA (2 x 64 + 64 ... the six 64-deep products per (q, key))
print(f"dK/dV' BH={BH} N={n}: {t:.3f} ms per launch ({fl / t / 1e9:.1f} TF/s at 6 x 2 x 64 FLOP per pair)", flush=True)
