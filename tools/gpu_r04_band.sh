#!/bin/bash
# Round 4 band passes: the all-zero-step skip of band strips (SGV_BAND_SKIP=0/1,
# product hashes must agree), then a kernel trace of the band passes (pack /
# MFMA / finalize split) at M = 1e6, bw = 1000, 8 and 16 columns.
#   bash tools/gpu_r04_band.sh <out-prefix>
set -o pipefail
out=$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "band" \
    --timeout 200 --timeout-method thread > ${out}_parity.log 2>&1 || { echo "band parity FAILED"; tail -30 ${out}_parity.log; exit 1; }
echo "band parity: $(tail -1 ${out}_parity.log)"
if [ -z "$BAND_TRACE_ONLY" ]; then
export SGV_AB=1
for rep in 1 2; do
  for v in 0 1; do
    SGV_BAND_SKIP=$v timeout -k 10 200 python -u tools/ldpass_band.py --tag "SGV_BAND_SKIP=$v" \
        --M 1000000 --bw 1000 --ncols 2,8,16 --reps 10 >> ${out}_ab.jsonl 2>> ${out}_ab.err || exit 1
  done
done
python3 -c "
import json
for l in open('${out}_ab.jsonl'):
    d = json.loads(l); print(d['tag'], d['ncol'], '%.4f ms' % d['ms_per_pass'], '%.3f' % d['frac_of_8TBs'], d['sha'])"
fi
R=$PWD
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/${out}_trace -o band --output-format csv -- \
    python3 -u $R/tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 8,16 --reps 10) > ${out}_trace.log 2>&1 || exit 1
f=$(find ${out}_trace -name "*kernel_stats.csv" | head -1)
cp "$f" ${out}_kernel_stats.csv
head -12 ${out}_kernel_stats.csv | cut -c1-200
