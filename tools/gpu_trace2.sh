#!/bin/bash
# Kernel + copy traces of bench.py for tools/step_timeline.py: C2's per-GPU
# share at N=8 (one LD block of 25,000) and C2 itself.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
T=${1:-r01}
tools/gpu_steps.sh \
  "b1tr_$T:300:cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/b1tr_$T -o run --output-format csv -- python3 $R/bench.py --blocks 1 --cpu-baseline off --steps 10" \
  "c2tr_$T:300:cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/c2tr_$T -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --steps 5 --warmup 2"
