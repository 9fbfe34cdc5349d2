"""Per-kernel time per step from a rocprofv3 kernel_trace.csv (--output-format csv).

usage: python tools/csvstats.py <run_kernel_trace.csv> [steps] [--grid]
--grid keeps launches with different grid sizes apart (tells GEMM/conv shapes apart)."""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
by_grid = "--grid" in sys.argv
steps = float(args[1]) if len(args) > 1 else 13.0
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(args[0])):
    k = r["Kernel_Name"][:90]
    if by_grid:
        k = (k, r.get("Grid_Size_X") or r.get("Grid_Size"))
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(v[1] for v in agg.values())
print(f"total kernel time {tot / steps:.3f} ms per step ({steps:g} steps)")
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    if t / steps < 0.01:
        continue
    print(f"  {t / steps:7.3f} ms/step  {n / steps:5.1f}/step  avg {t / n * 1e3:8.1f} us  {t / tot * 100:5.1f}%  {k}")
