#!/bin/bash
# Kernel traces of one bench config under SGV_STEP=phases (A) and the default (B)
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
ARGS=${AB_ARGS:---blocks 3 --block-size 7000 --steps 10 --warmup 2 --K 3 --ridge 0.1 --lmmse-damp 1}
tools/gpu_steps.sh \
  "trA:300:cd /tmp && SGV_STEP=phases rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/trA -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off $ARGS" \
  "trB:300:cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/trB -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off $ARGS"
