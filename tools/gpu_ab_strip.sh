#!/bin/bash
cd /root/repo || exit 2
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "ptest:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k 'strips or (ld_matvec_vs_numpy and packed) or shared_ld or 50_iter'" \
  "ab_c2_base:200:python tools/ldpass_bench.py --formats packed --ncols 2,3,4,8,12,16 --lib tools/ab/base.so" \
  "ab_c2_s8:200:python tools/ldpass_bench.py --formats packed --ncols 2,3,4,8,12,16" \
  "ab_c2_s4:200:SGV_MFMA_STRIP=4 python tools/ldpass_bench.py --formats packed --ncols 4,8,16" \
  "ab_c2_s16:200:SGV_MFMA_STRIP=16 python tools/ldpass_bench.py --formats packed --ncols 4,8,16" \
  "ab_m1e6_base:300:python tools/ldpass_bench.py --formats packed --blocks 64 --block-size 15625 --ncols 4,8,16 --lib tools/ab/base.so" \
  "ab_m1e6_s8:300:python tools/ldpass_bench.py --formats packed --blocks 64 --block-size 15625 --ncols 4,8,16" \
  "ab_m1e6_s4:300:SGV_MFMA_STRIP=4 python tools/ldpass_bench.py --formats packed --blocks 64 --block-size 15625 --ncols 4,8,16" \
  "ab_m1e6_s16:300:SGV_MFMA_STRIP=16 python tools/ldpass_bench.py --formats packed --blocks 64 --block-size 15625 --ncols 4,8,16"
