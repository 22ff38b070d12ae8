#!/bin/bash
# A/B of one A/B environment switch on bench.py (north-star default unless
# BENCH_ARGS is set), alternating runs of the same library:
#   tools/gpu_ab_env.sh TAG VAR VALUE   (B = SGV_AB=1 VAR=VALUE, A = default)
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=$1; VAR=$2; VAL=$3
mkdir -p gpurun_out
for rep in 1 2; do
for side in A B; do
  if [ $side = B ]; then envs="SGV_AB=1 $VAR=$VAL"; else envs=""; fi
  env $envs timeout -k 10 240 python bench.py --cpu-baseline off --steps 10 --warmup 3 $BENCH_ARGS \
      > "gpurun_out/${TAG}_${side}_$rep.log" 2>&1
  rc=$?
  echo "=== $side ($envs) rep $rep rc=$rc: $(grep '^{' gpurun_out/${TAG}_${side}_$rep.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("%.2f it/s %.2f ms/step pass %.3f ms frac %.4f launches %d" % (d["value"], d["ms_per_step"], r["avg_launch_ms"], r["frac"], r["launches"]))' 2>&1)"
  grep "^\[bench\] it=" "gpurun_out/${TAG}_${side}_$rep.log" | tail -3
  if [ $rc -ne 0 ]; then exit $rc; fi
done
done
