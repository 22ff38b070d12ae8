#!/bin/bash
# Round 4: how much the half-empty first item of band strips costs -- band
# passes at bandwidths whose stored extent is a whole number of 512-column
# chunks (bw 768: 1,024 columns; 1,280: 1,536) next to 1,000 (1,280 columns:
# every strip starts with a half-empty item), M = 1e6, 8 and 16 columns.
cd "$(dirname "$0")/.." || exit 2
tools/gpu_steps.sh \
  "bbw:600:for r in 1 2; do for bw in 768 1000 1280; do timeout -k 10 180 python -u tools/ldpass_band.py --tag bw\$bw --M 1000000 --bw \$bw --ncols 8,16 --reps 10 >> gpurun_out/bbw.jsonl || exit 1; done; done"
