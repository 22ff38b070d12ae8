#!/bin/bash
# Same-box A/B of the pipelined NC <= 2 packed pass (k_sym_pass_pl,
# SGV_SYM_PL=1) against k_sym_pass (default, SGV_SYM_PL=0): pass times, bench.py
# output files byte-identical between the two.
#   tools/gpu_ab_pl.sh
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "ld_matvec or ld_block or cg_solve" \
  > gpurun_out/pl_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -20 gpurun_out/pl_tests.log; exit 3; }
tail -1 gpurun_out/pl_tests.log
for rep in 1 2; do
  for v in 0 1; do
    echo "== C2 pl=$v"
    SGV_SYM_PL=$v timeout -k 10 200 python tools/ldpass_bench.py --formats packed_valu --ncols 1,2 --reps 20 || exit $?
  done
done
for v in 0 1; do
  echo "== M=1e6 pl=$v"
  SGV_SYM_PL=$v timeout -k 10 200 python tools/ldpass_bench.py --formats packed_valu --blocks 64 --block-size 15625 --ncols 1,2 --reps 5 || exit $?
done
W=$(mktemp -d /tmp/abpl.XXXX)
rc=0
for cfg in "k1:--blocks 2 --block-size 9000 --steps 6 --warmup 1" "b1:--blocks 1 --steps 20" "c2:--steps 10"; do
  n=${cfg%%:*}; args=${cfg#*:}
  for v in 0 1; do
    SGV_SYM_PL=$v timeout -k 10 200 python bench.py --cpu-baseline off --out-dir $W/$n$v $args \
      > gpurun_out/abpl_$n$v.log 2>&1 || { echo "[$n$v] bench failed rc=$?"; tail -5 gpurun_out/abpl_$n$v.log; exit 3; }
    echo "[$n pl=$v] $(tail -1 gpurun_out/abpl_$n$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f it/s %.3f ms/step pass %.3f ms" % (d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"]))')"
  done
  if diff -r -q $W/${n}0 $W/${n}1 > /dev/null; then
    echo "[$n] identical: $(ls $W/${n}0 | wc -l) files"
  else
    echo "[$n] DIFFER"; diff -r -q $W/${n}0 $W/${n}1 | head -5; rc=1
  fi
done
rm -rf $W
exit $rc
