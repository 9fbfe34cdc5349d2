"""One train_video.py step (VideoTrainer.step: forward, the temporal losses with the HIP warp and its
adjoint, backward, 3 Adam steps) at the script's shapes — 2 frame pairs of 256x512 with a 256x256
style (train_video.py:15-29, datasets.py:374-378) — timed with HIP events after warmup; synthetic
frames, a smooth random flow and a random consistency mask.

    python tools/video_train_time.py [steps] [warmup]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]

import torch  # noqa: E402

import network  # noqa: E402
from mhada_hip.recipe import load_recipe, seeded_image  # noqa: E402
from mhada_hip.train import VideoTrainer  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = "cuda"
    torch.manual_seed(0)
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(dev).train()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(dev).train()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").to(dev).train()
    vgg = load_recipe(network.VGG19(), "vgg").to(dev)
    tr = VideoTrainer(vc, vs, ada, vgg)
    B, H, W = 2, 256, 512
    style = seeded_image(B, 256, 256, 1).to(dev)
    c1 = seeded_image(B, H, W, 2).to(dev)
    c2 = seeded_image(B, H, W, 3).to(dev)
    yy, xx = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    flow = torch.stack([3 * torch.sin(yy / 17), 2 * torch.cos(xx / 23)]).unsqueeze(0).repeat(B, 1, 1, 1)
    mask = (torch.rand(B, H, W, device=dev) > 0.2).float()
    for _ in range(warmup):
        out = tr.step(style, c1, c2, flow, mask)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record()
    for _ in range(steps):
        out = tr.step(style, c1, c2, flow, mask)
    e.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    print(f"train_video step (B=2 frame pairs 256x512, style 256x256): {s.elapsed_time(e) / steps:.1f} ms/step "
          f"(wall {wall:.1f}); losses " + " ".join(f"{k} {v:.4g}" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    main()
