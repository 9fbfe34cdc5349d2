"""Per-config kernel time breakdown from a rocprofv3 kernel_trace.csv of bench.py.

usage: python tools/ktrace.py <run_kernel_trace.csv> [steps_per_config]
The bench runs the fp32 config first and the bf16 config second; the split point is the first
dispatch whose kernel name mentions bf16 (DF16b).  Times are per step (calls / steps)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13.0
split = next(i for i, r in enumerate(rows) if "DF16b" in r["Kernel_Name"] or "bf16" in r["Kernel_Name"])
for name, part in (("fp32 config", rows[:split]), ("bf16 config", rows[split:])):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in part:
        k = r["Kernel_Name"]
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot = sum(v[1] for v in agg.values())
    print(f"== {name}: {tot / steps:.2f} ms/step of kernel time ({steps:g} steps)")
    for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        if t / steps < 0.02:
            continue
        print(f"  {t / steps:7.3f} ms  {n / steps:5.1f}/step  avg {t / n * 1e3:8.1f} us  {k[:100]}")
