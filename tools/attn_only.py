"""Run only the bf16 (or fp32) MHAda attention kernel a few times (for rocprofv3 PMC passes).

    python tools/attn_only.py [bf16|f32|s3] [variant: fsq1 w8]   (s3: the fp32 SPLIT3 kernel)"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
from mhada_hip import _lib, ops

VARIANTS = {"fsq1": dict(attn_fixed_shift=1), "w8": dict(attn_fixed_shift=0)}
if len(sys.argv) > 2:
    for k, v in VARIANTS[sys.argv[2]].items():
        _lib.set_tuning(k, v)

s3 = len(sys.argv) > 1 and sys.argv[1] == "s3"
dt = torch.bfloat16 if (len(sys.argv) < 2 or sys.argv[1] == "bf16") else torch.float32
B, n = (4, 16384) if dt == torch.bfloat16 else (8, 4096)
H = 8
q = (torch.randn(B, H, n, 64, device="cuda") * 0.35).to(dt)
kv = (torch.randn(B, H, n, 128, device="cuda") * 0.35).to(dt)
vt = ops.transpose_v(kv)
fcs = torch.randn(B, n, 512, device="cuda")
mu, rs = ops.instnorm_stats(fcs)
vmu = torch.zeros(B, 512, device="cuda")
img = ops.split3_kv(kv, vt) if s3 else None
for _ in range(int(os.environ.get("ITERS", "5"))):
    if s3:
        ops.attn_split3(q, img, n, fcs, mu, rs, vmu)
    else:
        ops.mhada_attn(q, kv, vt, fcs, mu, rs, vmu, 0)
torch.cuda.synchronize()
print("done")
