#!/bin/bash
# Round 4: the NC = 5-8 MFMA kernel with and without the deferred row MFMAs
# (SGV_MF_DEFER=0; bitwise the same products): pass times on the north star,
# its 8-block share and C3's shape, then north-star bench lines, alternating.
cd "$(dirname "$0")/.." || exit 2
export SGV_AB=1
tools/gpu_steps.sh \
  "def_ab:700:for r in 1 2 3; do for v in 1 0; do SGV_MF_DEFER=\$v timeout -k 10 200 python -u tools/ldpass_ab.py --tag def\$v --shapes 64x15625,8x15625,8x25000 --ncols 6,8 --reps 10 >> gpurun_out/def_ab.jsonl || exit 1; done; done" \
  "def_bench:500:for r in 1 2; do for v in 1 0; do SGV_MF_DEFER=\$v timeout -k 10 200 python bench.py --cpu-baseline off --read-bw 0 | grep '^{' | sed \"s/^{/{\\\"variant\\\": \\\"def\$v\\\", /\" >> gpurun_out/def_bench.jsonl || exit 1; done; done"
