#!/bin/bash
# North-star configuration on one MI355X: M=1e6 in 64 LD blocks of 15,625,
# K=4 cohorts sharing the LD (8 CG columns on the MFMA pass), plus C4 (K=1)
# and C5 (K=8, s=0.1, damping, EM) at M=1e6, and the LD-pass microbenchmark
# at M=1e6 for 1/2/4/8 columns.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
T=${1:-r01}
M1E6="--blocks 64 --block-size 15625 --cpu-baseline off"
tools/gpu_steps.sh \
  "ns_k4_$T:300:python bench.py $M1E6 --K 4" \
  "c4_$T:300:python bench.py $M1E6 --K 1" \
  "c5_$T:300:python bench.py $M1E6 --K 8 --ridge 0.1 --lmmse-damp 1" \
  "ldp_m1e6_$T:300:python tools/ldpass_bench.py --blocks 64 --block-size 15625 --ncols 1,2,4,8 --formats packed"
