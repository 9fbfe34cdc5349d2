"""Average per-dispatch PMC counter values (summed over XCD/SE instances) for kernels whose
name contains a pattern.  usage: python tools/pmcsum.py <pattern> <counter_collection.csv>..."""
import collections
import csv
import sys

pat = sys.argv[1]
for f in sys.argv[2:]:
    agg = collections.defaultdict(float)
    durs = {}
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        durs[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per = collections.defaultdict(list)
    for (d, c), v in agg.items():
        per[c].append(v)
    print(f"{f}: {len(durs)} dispatches, avg {sum(durs.values()) / max(len(durs), 1):.1f} us")
    for c, v in sorted(per.items()):
        print(f"  {c:28s} {sum(v) / len(v):.4g}")
