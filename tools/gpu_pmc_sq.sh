#!/bin/bash
# SQ/GRBM counters (issue, waits, MFMA busy, clock) of the LD pass in the
# microbenchmark for prebuilt libraries: tools/gpu_pmc_sq.sh TAG NC lib1.so ...
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
TAG=$1; NC=$2; shift 2
mkdir -p gpurun_out
cd /tmp || exit 2
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/${TAG}_counters.txt" 2>&1
CNT=${CNT:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"}
for lib in "$@"; do
  n=$(basename "$lib" .so)
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d "$R/gpurun_out/${TAG}_$n" -o pmc --output-format csv -- \
    python3 "$R/tools/ldpass_bench.py" --lib "$R/$lib" --blocks 64 --block-size 15625 --ncols "$NC" \
    --formats packed --reps 3 > "$R/gpurun_out/${TAG}_$n.log" 2>&1
  rc=$?
  echo "=== $n rc=$rc"; tail -2 "$R/gpurun_out/${TAG}_$n.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
