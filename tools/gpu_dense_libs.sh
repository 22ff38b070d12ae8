#!/bin/bash
# Dense packed LD pass (ldpass_ab.py, product hashes) for the tree's build and
# each tools/ablib/libsgvamp_hip_<name>.so given, alternating twice.
#   bash tools/gpu_dense_libs.sh TAG name1 [name2 ...]
cd "$(dirname "$0")/.." || exit 2
T=$1; shift
o=gpurun_out/dlib_$T
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tree "$@"; do
    L=""; [ $lib != tree ] && L="--lib tools/ablib/libsgvamp_hip_$lib.so"
    timeout -k 10 300 python -u tools/ldpass_ab.py --tag "$lib" --shapes 64x15625,8x15625 \
        --ncols 4,8 $L >> $o.jsonl 2>> $o.err || exit 1
  done
done
python3 tools/ab_table.py $o.jsonl
