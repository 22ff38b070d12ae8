#!/bin/bash
# MFMA strip length (SGV_MFMA_STRIP, panels per strip) on the north-star block
# structure at the per-GPU shares of N = 1, 2, 4, 8 (64/32/16/8 blocks of 15,625),
# bench.py steps, alternating repeats in one call.
#   tools/gpu_strip_sweep.sh TAG "S1 S2 ..." "NBLK1 NBLK2 ..." [REPS]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=$1; SS=$2; BS=$3; REPS=${4:-2}
specs=()
for rep in $(seq 1 "$REPS"); do
  for B in $BS; do
    for S in $SS; do
      specs+=("${TAG}_b${B}_S${S}_r${rep}:200:SGV_AB=1 SGV_MFMA_STRIP=$S python bench.py --blocks $B --block-size 15625 --steps 10 --warmup 3 --cpu-baseline off")
    done
  done
done
tools/gpu_steps.sh "${specs[@]}"
