"""torch.profiler view of one train_image.py step (bench.py --train setup, 512^2 batch 8): device
time per aten / HIP-library op and, for the layout copies and adds, the Python call sites.
usage: python tools/train_torchprof.py [out.txt]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import network  # noqa: E402
from mhada_hip.recipe import load_recipe, seeded_image  # noqa: E402
from mhada_hip.train import Trainer  # noqa: E402

dev = torch.device("cuda")
vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(dev).train()
vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(dev).train()
ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").to(dev).train()
vgg = load_recipe(network.VGG19(), "vgg").to(dev)
tr = Trainer(vc, vs, ada, vgg)
imgs = [(seeded_image(8, 512, 512, 100 + i).to(dev), seeded_image(8, 512, 512, 500 + i).to(dev)) for i in range(3)]
for c, s in imgs[:2]:
    tr.step(c, s)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
    tr.step(*imgs[2])
    torch.cuda.synchronize()
out = open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout
print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=60), file=out)
for op in ("aten::copy_", "aten::add_", "aten::add", "aten::sum", "aten::mean", "aten::mul", "aten::sub",
           "aten::mse_loss", "aten::mse_loss_backward", "aten::std", "aten::div", "aten::cat"):
    rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key == op]
    rows.sort(key=lambda e: -e.self_device_time_total)
    print(f"\n==== {op}: top input shapes by device time", file=out)
    for e in rows[:15]:
        print(f"{e.self_device_time_total / 1e3:9.2f} ms  {e.count:5d} calls  {e.input_shapes}", file=out)
for op in ("aten::copy_", "aten::add", "aten::add_", "aten::cat", "aten::mse_loss_backward", "aten::fill_"):
    rows = [e for e in prof.key_averages(group_by_stack_n=6) if e.key == op]
    rows.sort(key=lambda e: -e.self_device_time_total)
    print(f"\n==== {op}: top call sites by device time", file=out)
    for e in rows[:12]:
        print(f"{e.self_device_time_total / 1e3:9.2f} ms  {e.count:5d} calls", file=out)
        for fr in e.stack[:6]:
            print(f"      {fr}", file=out)
