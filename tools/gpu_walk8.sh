#!/bin/bash
# Band walks up to 8 columns (SGV_AB=1 SGV_BAND_WALK=8): band parity suite with
# the walks forced, the pass microbenchmark alternating walks / strips at 3, 4
# and 8 columns, then the walkpmc counter passes.
#   bash tools/gpu_walk8.sh TAG
cd "$(dirname "$0")/.." || exit 2
T=${1:-w8}
o=gpurun_out/walk8_$T
mkdir -p gpurun_out
export TMPDIR=/tmp
SGV_AB=1 SGV_BAND_WALK=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_multirank.py -x -q -p no:cacheprovider -k "band or coupled or coupling" \
    --timeout 300 --timeout-method thread > $o.parity.log 2>&1 || { echo "parity FAILED"; tail -40 $o.parity.log; exit 1; }
tail -2 $o.parity.log
export SGV_AB=1
for rep in 1 2; do
  for v in 8 0; do
    SGV_BAND_WALK=$v timeout -k 10 300 python -u tools/ldpass_band.py --M 1000000 --bw 1000 \
        --ncols 3,4,8 --tag walk=$v >> $o.ab.jsonl 2>> $o.ab.err || exit 1
  done
done
python3 tools/ab_table.py $o.ab.jsonl
unset SGV_AB
bash tools/gpu_recipes.sh walkpmc $T
