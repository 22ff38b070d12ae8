#!/bin/bash
# A/B of the working-tree library against ab_lib/base.so (a build of another
# commit): bitwise results (tools/ab_bitwise.py) and LD-pass times, alternating.
#   tools/gpu_ab_lib.sh TAG NCOLS [extra ldpass_bench args]
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=$1; NC=$2; shift 2
MB="python tools/ldpass_bench.py --blocks 64 --block-size 15625 --formats packed --ncols $NC --reps 5 $*"
tools/gpu_steps.sh \
  "${TAG}_bitA:200:python tools/ab_bitwise.py --lib sgvamp-py_amd/libsgvamp_hip.so" \
  "${TAG}_bitB:200:python tools/ab_bitwise.py --lib ab_lib/base.so" \
  "${TAG}_mbA1:200:$MB" "${TAG}_mbB1:200:$MB --lib ab_lib/base.so" \
  "${TAG}_mbA2:200:$MB" "${TAG}_mbB2:200:$MB --lib ab_lib/base.so"
