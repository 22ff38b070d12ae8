#!/bin/bash
# One box's north-star bench line (default flags) and the same run with a
# one-rank RCCL communicator (the exchange's fixed cost); call repeatedly for
# the box-to-box spread.  bash tools/gpu_box_spread.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-a}
timeout -k 10 400 python -u bench.py --cpu-baseline off > gpurun_out/spread_${tag}.json 2> gpurun_out/spread_${tag}.err || exit 1
timeout -k 10 400 python -u bench.py --cpu-baseline off --exchange rccl > gpurun_out/spread_${tag}_rccl1.json 2> gpurun_out/spread_${tag}_rccl1.err || exit 1
python - <<PY
import json
for f in ("gpurun_out/spread_${tag}.json", "gpurun_out/spread_${tag}_rccl1.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, "it/s %.2f ms/step %.2f pass %.3f ms frac %.3f box %s" % (d["value"], d["ms_per_step"], r["avg_launch_ms"], r["frac"], r["box_stream_GBs"]))
PY
