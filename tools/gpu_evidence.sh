#!/bin/bash
# Round evidence on one MI355X: the default bench line (C2, with the CPU
# baseline), its kernel trace/stats, separate FETCH_SIZE / WRITE_SIZE passes
# for the dominant kernels at C2 (k_sym_pass) and C3 (k_sym_mfma), a C3 bench.
#   tools/gpu_evidence.sh TAG
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
T=${1:-r01}
A="--steps 5 --warmup 2 --cpu-baseline off"
tools/gpu_steps.sh \
  "bench_$T:300:python bench.py" \
  "trace_$T:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_$T -o bench --output-format csv -- python3 $R/bench.py $A" \
  "fetch_$T:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/fetch_$T -o pmc --output-format csv -- python3 $R/bench.py $A --no-files" \
  "write_$T:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/write_$T -o pmc --output-format csv -- python3 $R/bench.py $A --no-files" \
  "c3bench_$T:300:python bench.py --K 4 --cpu-baseline off" \
  "c3fetch_$T:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/c3fetch_$T -o pmc --output-format csv -- python3 $R/bench.py --K 4 $A --no-files" \
  "c3write_$T:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/c3write_$T -o pmc --output-format csv -- python3 $R/bench.py --K 4 $A --no-files"
