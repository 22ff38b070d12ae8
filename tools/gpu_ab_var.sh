#!/bin/bash
cd /root/repo || exit 2
for rep in 1 2; do
for nb in 8 4 2 1; do
for v in 0 2; do
  echo "nb=$nb var=$v"; SGV_SYM_VAR=$v timeout -k 10 100 python tools/ldpass_bench.py --formats packed --blocks $nb --ncols 1,2 --reps 20 || exit $?
done; done; done
for v in 0 2; do
  echo "nb=64x15625 var=$v"; SGV_SYM_VAR=$v timeout -k 10 100 python tools/ldpass_bench.py --formats packed --blocks 64 --block-size 15625 --ncols 1,2 --reps 5 || exit $?
done
