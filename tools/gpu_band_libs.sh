#!/bin/bash
# Band pass with the walks (SGV_BAND_WALK=8) for the tree's build and each
# tools/ablib/libsgvamp_hip_<name>.so given, alternating twice.
#   bash tools/gpu_band_libs.sh TAG name1 [name2 ...]
cd "$(dirname "$0")/.." || exit 2
T=$1; shift
o=gpurun_out/blib_$T
mkdir -p gpurun_out
export TMPDIR=/tmp SGV_AB=1 SGV_BAND_WALK=8
for rep in 1 2; do
  for lib in tree "$@"; do
    L=""; [ $lib != tree ] && L="--lib tools/ablib/libsgvamp_hip_$lib.so"
    timeout -k 10 300 python -u tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 3,4,8 \
        --tag "$lib" $L >> $o.jsonl 2>> $o.err || exit 1
  done
done
python3 tools/ab_table.py $o.jsonl
