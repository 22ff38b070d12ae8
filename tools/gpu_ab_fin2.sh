#!/bin/bash
# LD-pass A/B (same box): tools/ab/cur.so vs tools/ab/fin.so, M=1e6 and C2 sizes
cd "$(dirname "$0")/.." || exit 2
for lib in cur fin cur fin; do
  echo "== $lib M=1e6"; timeout -k 10 200 python tools/ldpass_bench.py --lib tools/ab/$lib.so --blocks 64 --block-size 15625 --ncols 4,8,16 --formats packed --reps 5 || exit $?
done
for lib in cur fin; do
  echo "== $lib C2"; timeout -k 10 200 python tools/ldpass_bench.py --lib tools/ab/$lib.so --ncols 4,8 --formats packed --reps 5 || exit $?
done
