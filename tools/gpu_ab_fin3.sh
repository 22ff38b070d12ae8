#!/bin/bash
# Finalize loops unrolled 4x (loads of four items in flight; same add order):
# bitwise A/B of bench outputs vs tools/ab/base.so, then pass times of both
# builds interleaved (C2 blocks NC 1/2/8, M=1e6 blocks NC 2/8).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
bash tools/gpu_ab_bitwise.sh || exit $?
steps=()
for i in 1 2; do
  for side in A B; do
    if [ $side = A ]; then L="--lib tools/ab/base.so"; else L=""; fi
    steps+=("fin_${side}${i}_c2:200:python tools/ldpass_bench.py $L --formats packed --ncols 1,2,8 --reps 5")
    steps+=("fin_${side}${i}_m1e6:200:python tools/ldpass_bench.py $L --formats packed --ncols 2,8 --reps 3 --blocks 64 --block-size 15625")
  done
done
tools/gpu_steps.sh "${steps[@]}"
