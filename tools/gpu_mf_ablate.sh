#!/bin/bash
# A/B of prebuilt variant libraries (gpu_variants/*.so) on the LD-pass microbenchmark
# at the north-star block structure (M=1e6, 64 x 15,625), NC from $NCS.
#   tools/gpu_mf_ablate.sh TAG lib1.so lib2.so ...
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=$1; shift
NCS=${NCS:-4,8}
mkdir -p gpurun_out
for rep in 1 2; do
for lib in "$@"; do
  n=$(basename "$lib" .so)
  echo "=== $n rep $rep"
  timeout -k 10 120 python tools/ldpass_bench.py --lib "$lib" --blocks 64 --block-size 15625 \
      --ncols "$NCS" --formats packed --reps 5 > "gpurun_out/${TAG}_${n}_$rep.log" 2>&1
  rc=$?
  cat "gpurun_out/${TAG}_${n}_$rep.log"
  if [ $rc -ne 0 ]; then echo "stop rc=$rc"; exit $rc; fi
done
done
