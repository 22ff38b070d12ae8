#!/bin/bash
# Kernel trace of the one-block configuration (C2's per-GPU share at N = 8)
# and of C2, for the per-step timeline (tools/step_timeline.py).
set -e
cd /root/repo
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /root/repo/gpurun_out/trb1 -o run -- python3 /root/repo/bench.py --cpu-baseline off --blocks 1 --steps 12 > /root/repo/gpurun_out/trb1.log 2>&1
cd /root/repo
python3 tools/step_timeline.py gpurun_out/trb1 --last 3 --gap-us 8
