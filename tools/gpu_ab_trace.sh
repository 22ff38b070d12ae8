#!/bin/bash
# A/B of the tree's library against ab_lib/base.so: bitwise results, then
# kernel traces of the LD-pass microbenchmark (per-kernel means per build).
#   tools/gpu_ab_trace.sh TAG NCOLS
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
TAG=$1; NC=$2
MB="$R/tools/ldpass_bench.py --blocks 64 --block-size 15625 --formats packed --ncols $NC --reps 5"
tools/gpu_steps.sh \
  "${TAG}_bitA:200:python tools/ab_bitwise.py --lib sgvamp-py_amd/libsgvamp_hip.so" \
  "${TAG}_bitB:200:python tools/ab_bitwise.py --lib ab_lib/base.so" \
  "${TAG}_trA:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trA -o mb --output-format csv -- python3 $MB" \
  "${TAG}_trB:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_trB -o mb --output-format csv -- python3 $MB --lib $R/ab_lib/base.so"
