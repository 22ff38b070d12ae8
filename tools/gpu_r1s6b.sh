#!/bin/bash
# Session-6 evidence, part 2: C4 and C5 on one GPU, PMC traffic of k_sym_mfma at
# the north-star configuration (M=1e6, K=4), the north-star kernel trace, smoke().
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
T=${1:-r01s6}
M1E6="--blocks 64 --block-size 15625 --cpu-baseline off"
A="$M1E6 --K 4 --steps 3 --warmup 2 --no-files"
tools/gpu_steps.sh \
  "smoke_$T:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "c4_$T:300:python bench.py $M1E6 --K 1" \
  "c5_$T:300:python bench.py $M1E6 --K 8 --ridge 0.1 --lmmse-damp 1 --steps 4" \
  "nstrace_$T:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/nstrace_$T -o ns --output-format csv -- python3 $R/bench.py $A" \
  "nsfetch_$T:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/nsfetch_$T -o pmc --output-format csv -- python3 $R/bench.py $A" \
  "nswrite_$T:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/nswrite_$T -o pmc --output-format csv -- python3 $R/bench.py $A"
