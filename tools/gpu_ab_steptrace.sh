#!/bin/bash
# A/B of the tree's library against ab_lib/base.so on whole bench steps, by
# kernel trace (GPU busy/idle time per step; tools/step_gaps.py reads them).
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
TAG=$1; shift
ARGS="--steps 10 --warmup 3 --cpu-baseline off $*"
cp sgvamp-py_amd/libsgvamp_hip.so /tmp/sgv_tree.so
tools/gpu_steps.sh \
  "${TAG}_trA:300:cd /tmp && cp /tmp/sgv_tree.so $R/sgvamp-py_amd/libsgvamp_hip.so && rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_trA -o st --output-format csv -- python3 $R/bench.py $ARGS" \
  "${TAG}_trB:300:cd /tmp && cp $R/ab_lib/base.so $R/sgvamp-py_amd/libsgvamp_hip.so && rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_trB -o st --output-format csv -- python3 $R/bench.py $ARGS"
cp /tmp/sgv_tree.so sgvamp-py_amd/libsgvamp_hip.so
