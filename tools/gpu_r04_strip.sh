#!/bin/bash
# Round 4: MFMA strip length 5 vs 8 panels (SGV_MFMA_STRIP; a different column-
# chain length, so different -- still N-invariant -- bits): the LPT model puts
# the 8-block share's launch at 0.986 of the perfect split with 5-panel strips
# (0.924 with 8) and the 64-block north star at 0.998 (0.994); measured on the
# north star, its 8- and 16-block shares and C3's shape at 4 / 8 / 16 columns.
cd "$(dirname "$0")/.." || exit 2
export SGV_AB=1
tools/gpu_steps.sh \
  "strip_ab:800:for r in 1 2 3; do for s in 8 5; do SGV_MFMA_STRIP=\$s timeout -k 10 250 python -u tools/ldpass_ab.py --tag S\$s --shapes 64x15625,8x15625,16x15625,8x25000 --ncols 4,8,16 --reps 10 >> gpurun_out/strip_ab.jsonl || exit 1; done; done" \
  "strip_bench:400:for r in 1 2; do for s in 8 5; do SGV_MFMA_STRIP=\$s timeout -k 10 150 python bench.py --cpu-baseline off --read-bw 0 | grep '^{' | sed \"s/^{/{\\\"variant\\\": \\\"S\$s\\\", /\" >> gpurun_out/strip_bench.jsonl || exit 1; done; done"
