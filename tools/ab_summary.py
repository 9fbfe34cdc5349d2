"""Summarise gpurun_out/ab_{on,off}_*.log (tools/gpu_ab_bench.sh): frames/s per config."""
import glob
import json

for tag in ("on", "off"):
    for f in sorted(glob.glob(f"gpurun_out/ab_{tag}_*.log")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        vals = [f"f32 {d['value']:.1f}"] + [f"{k} {v['value']:.1f}" for k, v in d.get("configs", {}).items()]
        print(tag, f[-5:-4], "  ".join(vals))
