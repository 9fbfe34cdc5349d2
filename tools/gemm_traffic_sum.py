"""Per-shape HBM traffic of tools/gemm_traffic_shapes.py from its rocprofv3 passes (tools/gemm_traffic.sh):
the GEMM dispatches in launch order, grouped per shape (1 warm-up + REPS launches, the warm-up dropped),
FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE against the algorithmic bytes the
shapes script prints, and the kernel-trace duration.

    python tools/gemm_traffic_sum.py gpurun_out/<tag>
"""
import csv
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_traffic_shapes import REPS  # noqa: E402


def gemm_rows(fn, key):
    rows = [r for r in csv.DictReader(open(fn)) if "gemm" in r["Kernel_Name"]]
    if key:
        rows = [r for r in rows if r["Counter_Name"] == key]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    return rows


def main():
    d = sys.argv[1]
    shapes = []
    for line in open(os.path.join(d, "fetch.log")):
        m = re.match(r"shape (\S+) algorithmic_read (\d+) algorithmic_write (\d+)", line)
        if m:
            shapes.append((m.group(1), int(m.group(2)), int(m.group(3))))
    f = gemm_rows(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = gemm_rows(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    t = [r for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))) if "gemm" in r["Kernel_Name"]]
    t.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = 1 + REPS
    # the split3 weight / row-split helpers are not GEMMs; the first GEMM launch belongs to the
    # script's m1 preparation (MLP1 -> planes) and precedes the measured shapes
    skip = len(f) - per * len(shapes)
    print(f"# GEMM dispatches: fetch {len(f)}, write {len(w)}, trace {len(t)}; leading non-measured {skip}")
    print("# traffic = FETCH_SIZE x 2 + WRITE_SIZE (KiB counters -> bytes); per launch, warm-up dropped")
    for i, (name, rd, wr) in enumerate(shapes):
        sl = slice(skip + i * per + 1, skip + (i + 1) * per)
        fb = [2 * float(r["Counter_Value"]) * 1024 for r in f[sl]]
        wb = [float(r["Counter_Value"]) * 1024 for r in w[sl]]
        ts = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in t[sl]]
        fa, wa, ta = sum(fb) / len(fb), sum(wb) / len(wb), sum(ts) / len(ts)
        kname = f[sl][0]["Kernel_Name"].split("(")[0][:60]
        print(f"{name:26s} {kname:60s} fetch {fa / 1e6:7.1f} MB (alg. read {rd / 1e6:7.1f}, x{fa / rd:.2f})  "
              f"write {wa / 1e6:7.1f} MB (alg. {wr / 1e6:6.1f}, x{wa / wr:.2f})  {ta:7.1f} us  "
              f"{(fa + wa) / ta / 1e6:.2f} TB/s")


if __name__ == "__main__":
    main()
