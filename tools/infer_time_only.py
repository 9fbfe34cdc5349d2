"""The reference's latency probe (infer_time.py:64-87) alone: B=1, 512^2, vit_c -> vit_s ->
adaFormer -> clamp, eager then hipGraph-replayed, N runs each (a target for rocprofv3 traces).
    python tools/infer_time_only.py [f32|bf16] [runs]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch

import bench
from mhada_hip.graphs import GraphedStylizer
from mhada_hip.recipe import seeded_image

dt = torch.bfloat16 if (len(sys.argv) > 1 and sys.argv[1] == "bf16") else torch.float32
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.cuda.set_device(0)
bench._DEVICE[0] = torch.device("cuda", 0)
vc, vs, ada = bench.build_models(dt)
c = seeded_image(1, 512, 512, 11).cuda()
s = seeded_image(1, 512, 512, 12).cuda()
with torch.no_grad():
    for _ in range(3):
        ada(vc(c), vs(s))[1].clamp(0, 255)
    torch.cuda.synchronize()
    for _ in range(runs):
        ada(vc(c), vs(s))[1].clamp(0, 255)
    torch.cuda.synchronize()
    g = GraphedStylizer(vc, vs, ada, (1, 3, 512, 512))
    for _ in range(runs):
        g(c, s)
    torch.cuda.synchronize()
print("done")
