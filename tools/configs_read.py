"""Table of tools/gpu_configs.sh bench lines (one row per configuration)."""
import json
import sys

tag = sys.argv[1]
for name in ("ns", "c2", "c3", "c4", "c5", "c5nd", "ns8blk"):
    try:
        line = [l for l in open("gpurun_out/%s_%s.log" % (name, tag)) if l.startswith("{")][-1]
    except (OSError, IndexError):
        print("%-7s missing" % name)
        continue
    d = json.loads(line)
    r = d["roofline"]
    print("%-7s %8.2f it/s %8.2f ms/step passes/step %.2f  ms/pass %.3f  frac %.3f  traffic %s" % (
        name, d["value"], d["ms_per_step"], d["ld_passes_per_step"], r["avg_launch_ms"],
        r["frac"], r.get("traffic_source")))
