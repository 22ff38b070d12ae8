#!/bin/bash
# Bench + profiles on the gpurun box:
#   kernel trace/stats (timing) and two separate --pmc passes (FETCH_SIZE, WRITE_SIZE).
#   tools/gpu_prof.sh TAG [extra bench.py args...]
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
TAG=${1:-r01}
shift
EXTRA="$*"
ARGS="--steps 5 --warmup 2 --cpu-baseline off $EXTRA"
tools/gpu_steps.sh \
  "bench_$TAG:300:python bench.py $EXTRA" \
  "trace_$TAG:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o bench --output-format csv -- python3 $R/bench.py $ARGS" \
  "pmc_fetch_$TAG:400:cd /tmp && rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv -- python3 $R/bench.py $ARGS --no-files" \
  "pmc_write_$TAG:400:cd /tmp && rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$TAG -o pmc --output-format csv -- python3 $R/bench.py $ARGS --no-files"
