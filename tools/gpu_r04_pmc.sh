#!/bin/bash
# Round 4: HBM traffic of the LD pass on the final tree (FETCH_SIZE and
# WRITE_SIZE in separate passes), north star and C5; summaries with
# tools/pmc_summary.py -> profiles/pmc_sym_mfma_r04_*.json
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
B="--steps 3 --warmup 1 --cpu-baseline off --read-bw 0"
C5="--K 8 --ridge 0.1 --lmmse-damp 1"
tools/gpu_steps.sh \
  "p4_ns_fetch:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/p4_ns_fetch -o pmc --output-format csv -- python3 $R/bench.py $B" \
  "p4_ns_write:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/p4_ns_write -o pmc --output-format csv -- python3 $R/bench.py $B" \
  "p4_c5_fetch:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/p4_c5_fetch -o pmc --output-format csv -- python3 $R/bench.py $B $C5" \
  "p4_c5_write:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/p4_c5_write -o pmc --output-format csv -- python3 $R/bench.py $B $C5"
