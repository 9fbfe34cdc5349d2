"""Per-kernel time summary from a rocprofv3 rocpd results.db (the ROCm 7 default output).
usage: python tools/dbstats.py <run_results.db> [steps] [--after NAME]
Prints total/avg per kernel name, sorted; `steps` divides totals into per-step figures."""
import collections
import sqlite3
import sys

db = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 1.0
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
agg = collections.defaultdict(lambda: [0, 0.0])
for name, s, e in rows:
    agg[name][0] += 1
    agg[name][1] += (e - s) / 1e6
tot = sum(v[1] for v in agg.values())
print(f"total kernel time {tot / steps:.3f} ms per step ({steps:g} steps, {len(rows)} dispatches)")
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    if t / steps < 0.005:
        continue
    print(f"{t / steps:8.3f} ms/step  {n / steps:6.1f}/step  avg {t / n * 1e3:9.1f} us  {100 * t / tot:5.1f}%  {k[:100]}")
