#!/bin/bash
# Session-6 evidence: GPU suite, default bench + kernel trace + PMC passes,
# C3 (K=4), one-block proxy, north-star M=1e6 K=4.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
T=${1:-r01s6}
A="--steps 5 --warmup 2 --cpu-baseline off"
tools/gpu_steps.sh \
  "gputests_$T:600:python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "bench_$T:300:python bench.py" \
  "trace_$T:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_$T -o bench --output-format csv -- python3 $R/bench.py $A" \
  "fetch_$T:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/fetch_$T -o pmc --output-format csv -- python3 $R/bench.py $A --no-files" \
  "write_$T:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/write_$T -o pmc --output-format csv -- python3 $R/bench.py $A --no-files" \
  "c3bench_$T:300:python bench.py --K 4 --cpu-baseline off" \
  "b1bench_$T:300:python bench.py --blocks 1 --cpu-baseline off --steps 20" \
  "nsk4_$T:300:python bench.py --blocks 64 --block-size 15625 --K 4 --cpu-baseline off"
