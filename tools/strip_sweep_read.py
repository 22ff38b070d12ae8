"""Table of tools/gpu_strip_sweep.sh results: avg LD-pass ms per (blocks, S)."""
import glob
import json
import os
import re
import sys
from collections import defaultdict

tag = sys.argv[1]
res = defaultdict(list)
for p in sorted(glob.glob("gpurun_out/%s_b*_S*_r*.log" % tag)):
    m = re.search(r"_b(\d+)_S(\d+)_r(\d+)\.log$", p)
    for line in open(p):
        if line.startswith("{") and '"value"' in line:
            d = json.loads(line)
            res[(int(m.group(1)), int(m.group(2)))].append(
                (d["roofline"]["avg_launch_ms"], d["ms_per_step"]))
for (b, s), v in sorted(res.items()):
    print("blocks %3d S %2d  pass ms %s  step ms %s" % (
        b, s, " ".join("%.4f" % x for x, _ in v), " ".join("%.3f" % y for _, y in v)))
