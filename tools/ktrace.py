"""Per-config kernel time breakdown from a rocprofv3 kernel_trace.csv of bench.py (--no-train).

usage: python tools/ktrace.py <run_kernel_trace.csv> [min_ms_per_step]
Configs are told apart by the MHAda attention launch grid (tools/attn_grid_stats.py CONFIGS);
every other kernel is assigned to the config of the next attention launch (the ViT and the
block projections precede it), so a config's decoder tail counts toward its next step.
Times are per step = per 6 attention launches (one per MHAda block)."""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from attn_grid_stats import CONFIGS  # noqa: E402

BY_GRID = {g: name for name, g in CONFIGS.items()}


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.02
    labels = [None] * len(rows)
    nxt = None
    for i in range(len(rows) - 1, -1, -1):
        r = rows[i]
        if "attn_" in r["Kernel_Name"] and "vit" not in r["Kernel_Name"] and "train" not in r["Kernel_Name"]:
            g = int(r["Grid_Size_X"])
            nxt = BY_GRID.get(g, nxt)
            if g in BY_GRID and "video" in nxt:
                nxt = nxt + (" bf16" if "bf16" in r["Kernel_Name"] else " f32")
        labels[i] = nxt
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
    nattn = collections.Counter()
    for r, lab in zip(rows, labels):
        if lab is None:
            continue
        k = r["Kernel_Name"]
        if "attn_" in k and "vit" not in k:
            nattn[lab] += 1
        per[lab][k][0] += 1
        per[lab][k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    for lab, agg in per.items():
        steps = nattn[lab] / 6.0
        tot = sum(v[1] for v in agg.values())
        print(f"== {lab}: {tot / steps:.3f} ms/step of kernel time ({steps:g} steps)")
        for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
            if t / steps < thr:
                continue
            print(f"  {t / steps:8.3f} ms  {n / steps:5.1f}/step  avg {t / n * 1e3:9.1f} us  {t / tot * 100:5.1f}%  {k[:96]}")


if __name__ == "__main__":
    main()
