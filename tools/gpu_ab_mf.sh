#!/bin/bash
cd /root/repo || exit 2
for rep in 1 2; do
for v in 0 1 2 3; do
  echo "C2 var=$v"; SGV_MF_VAR=$v timeout -k 10 100 python tools/ldpass_bench.py --formats packed --ncols 6,8 --reps 10 || exit $?
done; done
for v in 0 1 2; do
  echo "M1e6 var=$v"; SGV_MF_VAR=$v timeout -k 10 100 python tools/ldpass_bench.py --formats packed --blocks 64 --block-size 15625 --ncols 8 --reps 5 || exit $?
done
