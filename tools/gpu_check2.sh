#!/bin/bash
# GPU test suite, then traces of the one-block configuration (EM-heavy) and a
# C2 bench line, fused/unfused EM.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/gputests.log; exit 3; }
tail -1 gpurun_out/gputests.log
bash tools/gpu_trace_env.sh "--blocks 1 --steps 8" "SGV_EM_FUSE=1" "SGV_EM_FUSE=0" || exit $?
for v in 1 0; do
  SGV_EM_FUSE=$v timeout -k 10 200 python bench.py --cpu-baseline off --steps 10 > gpurun_out/c2_emf$v.log 2>&1 || exit $?
  echo "[c2 EM_FUSE=$v] $(grep '^{"metric' gpurun_out/c2_emf$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f it/s %.3f ms/step" % (d["value"], d["ms_per_step"]))')"
done
