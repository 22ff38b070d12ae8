#!/bin/bash
# A/B: finalize with 4 parts per row + largest-first item dispatch vs the previous build
cd /root/repo || exit 2
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "ptest:400:python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k 'strips or ld_matvec or golden or deterministic'" \
  "ab1_old:100:python tools/ldpass_bench.py --formats packed --blocks 1 --ncols 1,2,4,8 --reps 10 --lib tools/ab/strip.so" \
  "ab1_new:100:python tools/ldpass_bench.py --formats packed --blocks 1 --ncols 1,2,4,8 --reps 10" \
  "ab1_nolpt:100:SGV_SYM_LPT=0 python tools/ldpass_bench.py --formats packed --blocks 1 --ncols 1,2,4,8 --reps 10" \
  "ab8_old:100:python tools/ldpass_bench.py --formats packed --ncols 1,2,4,8 --reps 10 --lib tools/ab/strip.so" \
  "ab8_new:100:python tools/ldpass_bench.py --formats packed --ncols 1,2,4,8 --reps 10" \
  "ab8_nolpt:100:SGV_SYM_LPT=0 python tools/ldpass_bench.py --formats packed --ncols 1,2,4,8 --reps 10" \
  "bench:200:python bench.py --cpu-baseline off"
