#!/bin/bash
# A/B of two library builds (the tree's and tools/ablib/libsgvamp_hip_base.so):
# band parity with the walks forced to 8 columns and the packed LD-pass parity
# on the tree's build, then the band pass (walks and strips) and the dense
# packed pass, alternating builds twice (product hashes per build).
#   bash tools/gpu_lib_ab.sh TAG
cd "$(dirname "$0")/.." || exit 2
T=${1:-l}
o=gpurun_out/lib_$T
B=tools/ablib/libsgvamp_hip_base.so
mkdir -p gpurun_out
export TMPDIR=/tmp
SGV_AB=1 SGV_BAND_WALK=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_multirank.py -x -q -p no:cacheprovider -k "band or coupled or coupling" \
    --timeout 300 --timeout-method thread > $o.parity_walk8.log 2>&1 || { echo "walk8 parity FAILED"; tail -40 $o.parity_walk8.log; exit 1; }
tail -1 $o.parity_walk8.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider \
    -k "ld_matvec or mfma or band" --timeout 300 --timeout-method thread > $o.parity.log 2>&1 || { echo "parity FAILED"; tail -40 $o.parity.log; exit 1; }
tail -1 $o.parity.log
export SGV_AB=1
for rep in 1 2; do
  for lib in new base; do
    L=""; [ $lib = base ] && L="--lib $B"
    for v in 8 0; do
      SGV_BAND_WALK=$v timeout -k 10 300 python -u tools/ldpass_band.py --M 1000000 --bw 1000 \
          --ncols 3,4,8 --tag "$lib,walk=$v" $L >> $o.band_ab.jsonl 2>> $o.ab.err || exit 1
    done
    timeout -k 10 300 python -u tools/ldpass_ab.py --tag "$lib" --shapes 64x15625,8x15625 \
        --ncols 4,8 $L >> $o.dense_ab.jsonl 2>> $o.ab.err || exit 1
  done
done
python3 tools/ab_table.py $o.band_ab.jsonl
python3 tools/ab_table.py $o.dense_ab.jsonl
