#!/bin/bash
# A/B of the tree's library against ab_lib/base.so on the LD-pass microbenchmark at the
# north-star block structure, NC = 9/12/16 (the 16x16x4 / 4x4x4 C5 kernels), after the
# LD-pass parity tests; two alternating repeats.
cd /root/repo
export TMPDIR=/tmp
MB="tools/ldpass_bench.py --blocks 64 --block-size 15625 --formats packed --ncols 9,12,16 --reps 5"
tools/gpu_steps.sh \
  "lb_par:300:python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k 'ld_matvec_vs_numpy or mfma_strips or symmetry_and_linearity or band_vs_scipy'" \
  "lb_mbA1:200:python $MB" \
  "lb_mbB1:200:python $MB --lib ab_lib/base.so" \
  "lb_mbA2:200:python $MB" \
  "lb_mbB2:200:python $MB --lib ab_lib/base.so"
