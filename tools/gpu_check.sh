#!/bin/bash
# Full GPU test suite, then the same-box bitwise A/B against tools/ab/base.so
# (the previous build): every bench output file byte-identical, times beside.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/gputests.log; exit 3; }
tail -2 gpurun_out/gputests.log
bash tools/gpu_ab_bitwise.sh
