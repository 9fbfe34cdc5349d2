"""Same-process A/B of the headline inference step (bench.py configs[1]: vit_c, vit_s, adaFormer at
512^2 batch 8, fp32) under module-flag variants, interleaved rounds, median ms per step.

    python tools/infer_flags_ab.py "base:" "oproj32:ops.F32_SPLIT_OUTPROJ=0" [--rounds 7 --steps 10]
A variant is name:mod.FLAG=int,... with mod one of ops, engine (mhada_hip modules).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mhada-style-transfer_amd")]
import torch

import network
from mhada_hip import engine, ops
from mhada_hip.recipe import load_recipe, seeded_image

MODS = {"ops": ops, "engine": engine}


def parse(v):
    name, _, rest = v.partition(":")
    sets = []
    for item in filter(None, rest.split(",")):
        lhs, val = item.split("=")
        mod, attr = lhs.split(".")
        cur = getattr(MODS[mod], attr)
        sets.append((MODS[mod], attr, bool(int(val)) if isinstance(cur, bool) else int(val)))
    return name, sets


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    variants = [parse(v) for v in a.variants]
    dev = torch.device("cuda")
    vc = load_recipe(network.VisionTransformer(pos_embedding=True), "vit_c").to(dev).eval()
    vs = load_recipe(network.VisionTransformer(pos_embedding=False), "vit_s").to(dev).eval()
    ada = load_recipe(network.AdaAttnTransformerMultiHead(), "ada").to(dev).eval()
    c = seeded_image(a.batch, a.res, a.res, 1).to(dev)
    s = seeded_image(a.batch, a.res, a.res, 2).to(dev)

    def step():
        with torch.no_grad():
            return ada(vc(c), vs(s))[1]

    times = {n: [] for n, _ in variants}
    outs = {}
    for r in range(a.rounds + 1):
        for name, sets in variants:
            saved = [(m, at, getattr(m, at)) for m, at, _ in sets]
            for m, at, val in sets:
                setattr(m, at, val)
            try:
                torch.cuda.synchronize()
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                for _ in range(a.steps):
                    out = step()
                ev1.record()
                torch.cuda.synchronize()
                outs[name] = out
            finally:
                for m, at, val in saved:
                    setattr(m, at, val)
            if r > 0:
                times[name].append(ev0.elapsed_time(ev1) / a.steps)
        if r > 0:
            print(f"round {r}: " + "  ".join(f"{n} {times[n][-1]:.3f}" for n, _ in variants), flush=True)
    base = outs[variants[0][0]].double()
    for n, _ in variants:
        t = sorted(times[n])
        d = ((outs[n].double() - base).abs().max() / base.abs().max()).item()
        print(f"{n:10s} median {t[len(t) // 2]:.3f} ms/step  {a.batch * 1e3 / t[len(t) // 2]:.1f} frames/s  "
              f"(min {t[0]:.3f}, max {t[-1]:.3f})  max rel diff vs {variants[0][0]} {d:.2e}")


if __name__ == "__main__":
    main()
