#!/bin/bash
cd /root/repo || exit 2
for nb in 1 2 4 8; do
  for w in 1 0; do
    echo "blocks=$nb wide=$w"; SGV_SYM_WIDE=$w timeout -k 10 120 python tools/ldpass_bench.py --formats packed_valu --blocks $nb --ncols 1,2 --reps 10 || exit $?
  done
done
