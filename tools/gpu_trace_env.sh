#!/bin/bash
# Kernel traces of one bench configuration under several environments, one
# step timeline each (tools/step_timeline.py).  Usage:
#   tools/gpu_trace_env.sh "<bench args>" "ENV=1 ..." "ENV=0 ..." ...
set -e
cd /root/repo
export TMPDIR=/tmp
args=$1; shift
i=0
for v in "$@"; do
  i=$((i+1))
  echo "=== [$v] $args"
  (cd /tmp && env $v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/gpurun_out/trenv$i -o run -- python3 /root/repo/bench.py --cpu-baseline off $args > /root/repo/gpurun_out/trenv$i.log 2>&1)
  grep "^{\"metric" gpurun_out/trenv$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f it/s %.3f ms/step" % (d["value"], d["ms_per_step"]))'
  python3 tools/step_timeline.py gpurun_out/trenv$i --last 1 --gap-us 20 | head -24
done
