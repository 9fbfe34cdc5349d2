"""Training-step probe: per-step wall time with/without cudnn.benchmark (MIOpen find) and a
torch.profiler kernel breakdown of one steady-state step.
usage: python tools/train_probe.py [bench0|bench1] [prof]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch
import network
from mhada_hip.recipe import load_recipe, seeded_image
from mhada_hip.train import Trainer

torch.backends.cudnn.benchmark = "bench1" in sys.argv
dev = torch.device("cuda")
vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(dev).train()
vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(dev).train()
ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").to(dev).train()
vgg = load_recipe(network.VGG19(), "vgg").to(dev)
tr = Trainer(vc, vs, ada, vgg)
c = seeded_image(8, 512, 512, 100).to(dev)
s = seeded_image(8, 512, 512, 500).to(dev)
for i in range(5):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    tr.step(c, s)
    torch.cuda.synchronize(); print(f"step {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
if "prof" in sys.argv:
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CUDA]) as p:
        tr.step(c, s)
        torch.cuda.synchronize()
    print(p.key_averages().table(sort_by="cuda_time_total", row_limit=25, max_name_column_width=70))
