"""Per-config kernel time breakdown from a rocprofv3 kernel_trace.csv of bench.py (--no-train).

usage: python tools/ktrace.py <run_kernel_trace.csv> [min_ms_per_step] [--markers=<run_marker_api_trace.csv>]
                              [--bench=<stdout of the profiled bench.py>]
With --bench (round 6): each config's line also carries the shader clock that the SAME profiled process
measured right after that config's timed region (bench.py shader_clock, the "clock_ghz" of its JSON
line) and the bench's own HIP-event attention average, so the trace's attention average and the
roofline fraction of any bench line can be compared at a known clock.
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


def bench_info(fn):
    """{config: (clock_ghz, attention avg_launch_ms or None)} from the JSON line of a bench.py log."""
    import json
    line = [ln for ln in open(fn) if ln.startswith("{")][-1]
    d = json.loads(line)
    out = {"512x512_b8_f32": (d.get("clock_ghz"), d.get("roofline", {}).get("avg_launch_ms"))}
    for k, v in d.get("configs", {}).items():
        key = {"1024x1024_b4_bf16": "1024x1024_b4_bf16"}.get(k, k.replace("_s256", ""))
        out[key] = (v.get("clock_ghz"), (v.get("roofline") or {}).get("avg_launch_ms"))
    return out


def by_markers(rows, ranges, thr, bench=None):
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
        if bench and cfg in bench:
            clk, ev = bench[cfg]
            att = [(n, t) for k, (n, t) in agg.items() if "attn_" in k and "vit" not in k]
            line = f"  clock {clk} GHz (shader clock measured by this profiled process after the timed region)"
            if att and ev:
                tr = sum(t for _, t in att) / sum(n for n, _ in att)
                line += f"; attention trace avg {tr * 1e3:.1f} us vs the bench's HIP events {ev * 1e3:.1f} us ({tr / ev - 1:+.1%})"
            print(line)


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    args = [a for a in sys.argv[2:] if not a.startswith("--")]
    thr = float(args[0]) if args else 0.02
    mk = [a.split("=", 1)[1] for a in sys.argv[2:] if a.startswith("--markers=")]
    bk = [a.split("=", 1)[1] for a in sys.argv[2:] if a.startswith("--bench=")]
    if mk:
        return by_markers(rows, marker_ranges(mk[0]), thr, bench_info(bk[0]) if bk else None)
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
