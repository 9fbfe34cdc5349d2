"""Average duration of the MHAda attention kernel per bench config from a rocprofv3
kernel_trace.csv of the default bench command (configs told apart by grid size), to set beside
the bench line's roofline.avg_launch_ms (HIP events on the launch stream).

usage: python tools/attn_grid_stats.py <run_kernel_trace.csv>
"""
import collections
import csv
import sys

# grid size (threads, X) per bench config: blocks = B*H*ceil(Nc/256), 512 threads each
CONFIGS = {"512x512_b8_f32": 8 * 8 * (4096 // 256) * 512,
           "1024x1024_b4_bf16": 4 * 8 * (16384 // 256) * 512,
           "video_1080p (Nc=32400, Ns=1024)": 1 * 8 * ((32400 + 255) // 256) * 512}


def main():
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"]
        if "attn_" not in name or "vit" in name:
            continue
        d[(int(r["Grid_Size_X"]), name.split("(")[0])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for cfg, grid in CONFIGS.items():
        for (g, name), v in sorted(d.items()):
            if g == grid:
                print(f"{cfg:32s} {name:42s} launches {len(v):4d}  avg {sum(v) / len(v):.4f} ms  "
                      f"min {min(v):.4f}  max {max(v):.4f}")


if __name__ == "__main__":
    main()
