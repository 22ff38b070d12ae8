#!/bin/bash
# A/B of the tree's library against ab_lib/base.so on whole bench steps: the
# library file is swapped in place on the box (the box's copy of the tree only).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=$1; shift
ARGS="$* --cpu-baseline off"
cp sgvamp-py_amd/libsgvamp_hip.so /tmp/sgv_tree.so
tools/gpu_steps.sh \
  "${TAG}_bitA:200:python tools/ab_bitwise.py --lib sgvamp-py_amd/libsgvamp_hip.so" \
  "${TAG}_bitB:200:python tools/ab_bitwise.py --lib ab_lib/base.so" \
  "${TAG}_A1:300:cp /tmp/sgv_tree.so sgvamp-py_amd/libsgvamp_hip.so && python bench.py $ARGS" \
  "${TAG}_B1:300:cp ab_lib/base.so sgvamp-py_amd/libsgvamp_hip.so && python bench.py $ARGS" \
  "${TAG}_A2:300:cp /tmp/sgv_tree.so sgvamp-py_amd/libsgvamp_hip.so && python bench.py $ARGS" \
  "${TAG}_B2:300:cp ab_lib/base.so sgvamp-py_amd/libsgvamp_hip.so && python bench.py $ARGS"
cp /tmp/sgv_tree.so sgvamp-py_amd/libsgvamp_hip.so
