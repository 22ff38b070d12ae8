#!/bin/bash
# Roofline evidence for one bench workload: a kernel trace of the bench command
# (pass times vs the bench line's HIP events: trace_pass_summary.py), then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (pmc_summary.py).
#   tools/gpu_evidence.sh TAG [bench.py args...]
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
TAG=${1:-r03}
shift
ARGS="--steps 5 --warmup 2 --cpu-baseline off --read-bw 0 $*"
tools/gpu_steps.sh \
  "trace_$TAG:400:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o bench --output-format csv -- python3 $R/bench.py $ARGS" \
  "pmc_fetch_$TAG:300:cd /tmp && timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv -- python3 $R/bench.py $ARGS --no-files" \
  "pmc_write_$TAG:300:cd /tmp && timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$TAG -o pmc --output-format csv -- python3 $R/bench.py $ARGS --no-files"
