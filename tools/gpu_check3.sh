#!/bin/bash
# Multi-rank / exchange tests, then the exchange path's cost on the one-block
# configuration: no communicator vs one-rank RCCL communicator (replicated EM
# on / off).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_cli.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/mr_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/mr_tests.log; exit 3; }
tail -1 gpurun_out/mr_tests.log
for cfg in "none:" "rccl:--exchange rccl" "rccl_norep:--exchange rccl" "host:--exchange host"; do
  n=${cfg%%:*}; args=${cfg#*:}
  env=""; [ $n = rccl_norep ] && env="SGV_EM_REP=0"
  env $env timeout -k 10 200 python bench.py --cpu-baseline off --blocks 1 --steps 10 $args > gpurun_out/ex_$n.log 2>&1 || { echo "[$n] failed"; tail -5 gpurun_out/ex_$n.log; exit 3; }
  echo "[b1 $n] $(grep '^{"metric' gpurun_out/ex_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f it/s %.3f ms/step" % (d["value"], d["ms_per_step"]))')"
done
