#!/bin/bash
# A/B of prebuilt libraries on bench.py (north-star default unless BENCH_ARGS
# is set): each library is copied over the in-tree build for its run, and the
# in-tree build is restored at the end.  tools/gpu_bench_ab.sh TAG lib1.so ...
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
TAG=$1; shift
LIB=sgvamp-py_amd/libsgvamp_hip.so
cp "$LIB" /tmp/libsgvamp_hip.orig.so
mkdir -p gpurun_out
rc=0
for rep in 1 2; do
for lib in "$@"; do
  n=$(basename "$lib" .so)
  cp "$lib" "$LIB"
  timeout -k 10 240 python bench.py --cpu-baseline off --steps 10 --warmup 3 $BENCH_ARGS \
      > "gpurun_out/${TAG}_${n}_$rep.log" 2>&1
  rc=$?
  echo "=== $n rep $rep rc=$rc: $(tail -1 gpurun_out/${TAG}_${n}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("%.2f it/s pass %.3f ms frac %.4f" % (d["value"], r["avg_launch_ms"], r["frac"]))' 2>&1)"
  if [ $rc -ne 0 ]; then break 2; fi
done
done
cp /tmp/libsgvamp_hip.orig.so "$LIB"
exit $rc
