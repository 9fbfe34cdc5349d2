"""Per-kernel time over the last `ms` milliseconds of a rocprofv3 kernel trace (the steady-state
step of a run whose first steps include library tuning).
usage: python tools/laststep.py <kernel_trace.csv> <ms> [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
span = float(sys.argv[2]) * 1e6
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
st = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
end = st[-1][1]
win = [x for x in st if x[0] > end - span]
tot = sum(e - s for s, e, _ in win)
print(f"window: {len(win)} kernels, busy {tot / 1e6:.2f} ms over {(end - win[0][0]) / 1e6:.2f} ms")
agg = collections.defaultdict(lambda: [0, 0])
for s, e, n in win:
    agg[n[:100]][0] += e - s
    agg[n[:100]][1] += 1
for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
    print(f"{t / 1e6:8.2f} ms {c:5d}  {n}")
