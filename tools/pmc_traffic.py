"""Per-launch HBM traffic of the MHAda attention kernel from rocprofv3 PMC passes.

    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports exactly half the bytes of a wide
coalesced streaming read on gfx950 -> doubled; WRITE_SIZE (KiB) is exact for 16-B stores.  The two
counters come from separate passes (they cannot share one).  Keyed by bench config via grid size.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import attn_source_sha  # noqa: E402

# grid size (threads) of mhada_attn per bench config: blocks = B*H*ceil(Nc/256), 512 threads each
CONFIGS = {"512x512_b8_f32": 8 * 8 * (4096 // 256) * 512, "1024x1024_b4_bf16": 4 * 8 * (16384 // 256) * 512}


NAMES = {}  # grid size -> the attention kernel's name (attn_s3_kernel for the fp32 SPLIT3 path, round 6)


def load(fn, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(fn)):
        if "attn_" in r["Kernel_Name"] and "vit" not in r["Kernel_Name"] and r["Counter_Name"] == counter:
            d[int(r["Grid_Size"])].append(float(r["Counter_Value"]))
            NAMES[int(r["Grid_Size"])] = r["Kernel_Name"].split("(")[0].replace("void ", "")
    return d


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    out = {"attn_src_sha": attn_source_sha()}
    for name, grid in CONFIGS.items():
        if grid not in f or grid not in w:
            continue
        fetch = 2.0 * 1024 * sum(f[grid]) / len(f[grid])
        write = 1024.0 * sum(w[grid]) / len(w[grid])
        out[name] = {"kernel": NAMES.get(grid, "mhada_attn"), "launches": len(f[grid]), "fetch_bytes_corrected": fetch,
                     "write_bytes": write, "traffic_bytes_per_launch": fetch + write,
                     "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; separate --pmc passes"}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
