#!/bin/bash
# PMC traffic (FETCH_SIZE and WRITE_SIZE, separate passes) of the LD pass at
# C4 (M=1e6, K=1: k_sym_pass) and C5 (M=1e6, K=8: k_sym_mfma16).
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
M1E6="--blocks 64 --block-size 15625 --cpu-baseline off --steps 3 --warmup 1 --no-files"
C5="$M1E6 --K 8 --ridge 0.1 --lmmse-damp 1"
tools/gpu_steps.sh \
  "c4fetch:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/c4fetch -o pmc --output-format csv -- python3 $R/bench.py $M1E6" \
  "c4write:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/c4write -o pmc --output-format csv -- python3 $R/bench.py $M1E6" \
  "c5fetch:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/c5fetch -o pmc --output-format csv -- python3 $R/bench.py $C5" \
  "c5write:300:cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/c5write -o pmc --output-format csv -- python3 $R/bench.py $C5"
