#!/bin/bash
# Same-box A/B of two library builds: every output file (.bin trajectories and
# CSVs) of bench.py runs must be byte-identical, and the step logs' CG/EM counts
# equal.  A = tools/ab/base.so (the previous build), B = the tree's library.
#   tools/gpu_ab_bitwise.sh
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
W=$(mktemp -d /tmp/abbit.XXXX)
rc=0
run() {   # name args...
  local n=$1; shift
  for side in A B; do
    if [ $side = A ]; then lib=${AB_LIB_A-tools/ab/base.so}; stp=${AB_STEP_A:-}; else lib=; stp=; fi
    SGV_STEP=$stp SGV_LIB=$lib timeout -k 10 200 python bench.py --cpu-baseline off --out-dir $W/$n$side "$@" \
      > gpurun_out/ab_$n$side.log 2>&1 || { echo "[$n$side] bench failed rc=$?"; tail -5 gpurun_out/ab_$n$side.log; exit 3; }
  done
  if diff -r -q $W/${n}A $W/${n}B > /dev/null; then
    echo "[$n] identical: $(ls $W/${n}A | wc -l) files"
  else
    echo "[$n] DIFFER"; diff -r -q $W/${n}A $W/${n}B | head -5; rc=1
  fi
  diff <(grep -o 'cg=.*em=[0-9]*' gpurun_out/ab_${n}A.log) <(grep -o 'cg=.*em=[0-9]*' gpurun_out/ab_${n}B.log) > /dev/null \
    && echo "[$n] same CG/EM counts" || { echo "[$n] CG/EM counts differ"; rc=1; }
  for side in A B; do
    echo "[$n$side] $(tail -1 gpurun_out/ab_$n$side.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f it/s %.3f ms/step" % (d["value"], d["ms_per_step"]))')"
  done
}
run k1   --blocks 2 --block-size 9000 --steps 6 --warmup 1
run k4   --blocks 2 --block-size 9000 --steps 6 --warmup 1 --K 4
run k3sd --blocks 3 --block-size 7000 --steps 6 --warmup 1 --K 3 --ridge 0.1 --lmmse-damp 1
run b1   --blocks 1 --steps 20
run c2   --steps 10
rm -rf $W
exit $rc
