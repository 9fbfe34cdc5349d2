"""Summarise a rocprofv3 kernel_stats.csv: per-kernel total/avg time, sorted.
usage: python tools/kstats.py gpurun_out/prof/<name>_kernel_stats.csv [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / steps:.2f} ms per step ({steps:g} steps)")
for r in rows:
    t = float(r["TotalDurationNs"]) / 1e6 / steps
    if t < 0.01:
        continue
    print(f"{t:8.3f} ms/step  calls/step {int(r['Calls']) / steps:6.1f}  avg {float(r['AverageNs']) / 1e3:9.1f} us  "
          f"{float(r['Percentage']):5.1f}%  {r['Name'][:110]}")
