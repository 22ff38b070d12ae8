#!/bin/bash
# Round evidence without PMC passes: default bench line (C2 + CPU baseline),
# its kernel trace/stats, C3 (K=4), the one-block per-rank proxy of N=8, and the
# north-star configuration (M=1e6, K=4) on one GPU.
#   tools/gpu_round.sh TAG
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
T=${1:-r01}
tools/gpu_steps.sh \
  "bench_$T:300:python bench.py" \
  "trace_$T:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_$T -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline off" \
  "c3bench_$T:300:python bench.py --K 4 --cpu-baseline off" \
  "b1bench_$T:300:python bench.py --blocks 1 --cpu-baseline off --steps 20" \
  "nsk4_$T:300:python bench.py --blocks 64 --block-size 15625 --K 4 --cpu-baseline off"
