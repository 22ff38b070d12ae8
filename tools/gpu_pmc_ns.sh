#!/bin/bash
# North-star bench: kernel trace, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
TAG=${1:-r02}
ARGS="--steps 5 --warmup 2 --cpu-baseline off"
tools/gpu_steps.sh \
  "trace_$TAG:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o bench --output-format csv -- python3 $R/bench.py $ARGS" \
  "pmc_fetch_$TAG:300:cd /tmp && timeout -s KILL 250 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv -- python3 $R/bench.py $ARGS --no-files" \
  "pmc_write_$TAG:300:cd /tmp && timeout -s KILL 250 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$TAG -o pmc --output-format csv -- python3 $R/bench.py $ARGS --no-files"
