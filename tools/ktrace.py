"""Per-config kernel time breakdown from a rocprofv3 kernel_trace.csv of bench.py (--no-train).

usage: python tools/ktrace.py <run_kernel_trace.csv> [min_ms_per_step] [--markers=<run_marker_api_trace.csv>]
With --markers (rocprofv3 --marker-trace): the bench's roctx ranges bound each config's timed
region exactly (round 4).  Without: configs are told apart by the MHAda attention launch grid (tools/attn_grid_stats.py CONFIGS);
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


def marker_ranges(fn):
    """bench.py's roctx ranges "bench:<config>:<steps>" from a rocprofv3 marker_api_trace.csv:
    [(config, steps, start_ns, end_ns)]."""
    out = []
    for r in csv.DictReader(open(fn)):
        text = next((v for v in r.values() if isinstance(v, str) and v.startswith("bench:")), None)
        if text is None:
            continue
        _, cfg, steps = text.split(":")
        out.append((cfg, int(steps), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def by_markers(rows, ranges, thr):
    """Kernels whose execution lies inside a config's timed region, per timed step: every launch of
    a timed region is counted once and nothing outside it (warm-up, other configs) leaks in."""
    for cfg, steps, t0, t1 in ranges:
        agg = collections.defaultdict(lambda: [0, 0.0])
        first = last = None
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s < t0 or e > t1:
                continue
            first = s if first is None else min(first, s)
            last = e if last is None else max(last, e)
            agg[r["Kernel_Name"]][0] += 1
            agg[r["Kernel_Name"]][1] += (e - s) / 1e6
        if not agg:
            continue
        tot = sum(v[1] for v in agg.values())
        wall = (last - first) / 1e6
        print(f"== {cfg}: {tot / steps:.3f} ms/step of kernel time, {wall / steps:.3f} ms/step from the first kernel's "
              f"start to the last one's end ({steps} timed steps; kernel time / span = {tot / wall:.3f})")
        for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
            if t / steps < thr:
                continue
            print(f"  {t / steps:8.3f} ms  {n / steps:5.1f}/step  avg {t / n * 1e3:9.1f} us  {t / tot * 100:5.1f}%  {k[:96]}")


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    args = [a for a in sys.argv[2:] if not a.startswith("--markers=")]
    thr = float(args[0]) if args else 0.02
    mk = [a.split("=", 1)[1] for a in sys.argv[2:] if a.startswith("--markers=")]
    if mk:
        return by_markers(rows, marker_ranges(mk[0]), thr)
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
