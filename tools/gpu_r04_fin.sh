#!/bin/bash
# Round 4: the finalize with one thread per panel row (SGV_FIN_FORM=1, bitwise the
# same outputs) and band plans' prefetch depth 4 (SGV_BAND_PD=4) against the
# defaults: band M = 1e6, bw = 1,000 at 8 / 16 columns, dense north star and its
# 8-block share at 8 columns, C5's 16.  Product hashes must agree per shape.
#   bash tools/gpu_r04_fin.sh <out-prefix>
set -o pipefail
out=$1
export SGV_AB=1
SGV_FIN_FORM=1 SGV_BAND_PD=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "band or strips or coupled" --timeout 200 --timeout-method thread > ${out}_parity.log 2>&1 \
    || { echo "parity FAILED"; tail -30 ${out}_parity.log; exit 1; }
echo "parity (FIN_FORM=1, BAND_PD=4): $(tail -1 ${out}_parity.log)"
for rep in 1 2; do
  for v in "4 2" "1 2" "1 4" "4 4"; do
    set -- $v
    SGV_FIN_FORM=$1 SGV_BAND_PD=$2 timeout -k 10 200 python -u tools/ldpass_band.py \
        --tag "fin=$1 pd=$2" --M 1000000 --bw 1000 --ncols 8,16 --reps 10 >> ${out}_band.jsonl \
        2>> ${out}_ab.err || exit 1
  done
  for f in 4 1; do
    SGV_FIN_FORM=$f timeout -k 10 200 python -u tools/ldpass_ab.py --tag "fin=$f" \
        --shapes 64x15625,8x15625 --ncols 8,16 --reps 10 >> ${out}_dense.jsonl 2>> ${out}_ab.err || exit 1
  done
done
python3 -c "
import json
for f in ('${out}_band.jsonl', '${out}_dense.jsonl'):
    for l in open(f):
        d = json.loads(l)
        print(d['tag'], d.get('shape', d.get('bw')), d['ncol'], '%.4f ms' % d['ms_per_pass'],
              '%.3f' % d.get('frac_of_8TBs', d.get('stored_GBs', 0) / 8000), d['sha'])"
