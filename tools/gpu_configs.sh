#!/bin/bash
# Every BASELINE.json configuration that fits one MI355X, on the current tree:
# the north star (the bench line), C2, C3, C4 and C5 (as configured and without
# damping), plus the N = 8 per-GPU share of the north star (8 blocks).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
T=${1:-cfg}
M1E6="--blocks 64 --block-size 15625 --cpu-baseline off --steps 20 --warmup 3"
M2E5="--blocks 8 --block-size 25000 --cpu-baseline off --steps 20 --warmup 3"
tools/gpu_steps.sh \
  "ns_$T:300:python bench.py $M1E6 --K 4" \
  "c2_$T:300:python bench.py $M2E5 --K 1" \
  "c3_$T:300:python bench.py $M2E5 --K 4" \
  "c4_$T:300:python bench.py $M1E6 --K 1" \
  "c5_$T:300:python bench.py $M1E6 --K 8 --ridge 0.1 --lmmse-damp 1" \
  "c5nd_$T:300:python bench.py $M1E6 --K 8 --ridge 0.1" \
  "ns8blk_$T:300:python bench.py --blocks 8 --block-size 15625 --cpu-baseline off --steps 20 --warmup 3 --K 4"
