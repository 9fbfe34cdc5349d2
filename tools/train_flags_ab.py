"""Same-process A/B of the 512^2 B8 training step (bench.py --train's Trainer and data) under
module-flag variants, interleaved rounds of a few steps each, median ms per step — box-to-box clock
differences (several ms per step) otherwise hide changes of a few ms.

    python tools/train_flags_ab.py "base:" "dq32:ops.TRAIN_DQ_S3=0" [--rounds 5 --steps 3]
A variant is name:mod.FLAG=int,... with mod one of ops, train_fns, engine (mhada_hip modules).
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

import network
from mhada_hip import engine, ops, train_fns
from mhada_hip.recipe import load_recipe, seeded_image
from mhada_hip.train import Trainer

MODS = {"ops": ops, "train_fns": train_fns, "engine": engine}


def parse(v):
    name, _, rest = v.partition(":")
    sets = []
    for item in filter(None, rest.split(",")):
        lhs, val = item.split("=")
        mod, attr = lhs.split(".")
        sets.append((MODS[mod], attr, bool(int(val)) if isinstance(getattr(MODS[mod], attr), bool) else int(val)))
    return name, sets


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    variants = [parse(v) for v in a.variants]
    dev = torch.device("cuda")
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(dev).train()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(dev).train()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").to(dev).train()
    vgg = load_recipe(network.VGG19(), "vgg").to(dev)
    tr = Trainer(vc, vs, ada, vgg)
    data = [(seeded_image(8, 512, 512, 100 + i).to(dev), seeded_image(8, 512, 512, 500 + i).to(dev))
            for i in range(a.steps)]
    times = {n: [] for n, _ in variants}
    for r in range(a.rounds + 1):
        for name, sets in variants:
            saved = [(m, at, getattr(m, at)) for m, at, _ in sets]
            for m, at, val in sets:
                setattr(m, at, val)
            try:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for c, s in data:
                    tr.step(c, s)
                torch.cuda.synchronize()
                el = (time.perf_counter() - t0) / a.steps * 1e3
            finally:
                for m, at, val in saved:
                    setattr(m, at, val)
            if r > 0:  # round 0 warms every variant up
                times[name].append(el)
        if r > 0:
            print(f"round {r}: " + "  ".join(f"{n} {times[n][-1]:.1f}" for n, _ in variants), flush=True)
    for n, _ in variants:
        t = sorted(times[n])
        print(f"{n:10s} median {t[len(t) // 2]:.2f} ms/step  (min {t[0]:.2f}, max {t[-1]:.2f})")


if __name__ == "__main__":
    main()
