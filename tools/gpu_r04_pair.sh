#!/bin/bash
# Round 4: the wave-pair MFMA kernel (k_sym_mfma_pair) against the 4-wave one --
# bitwise test, LD-pass A/B with product hashes on the north star's block shape
# at 64 / 16 / 8 blocks and C3's, then bench lines of the 8-block share and the
# north star with the plan's choice forced each way (SGV_MF_PAIR=0/1).
#   bash tools/gpu_r04_pair.sh <out-prefix>
set -o pipefail
out=$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mfma_pair_kernel_bitwise or mfma_strips_vs_numpy" \
    --timeout 200 --timeout-method thread > ${out}_tests.log 2>&1 || { echo "tests FAILED"; tail -30 ${out}_tests.log; exit 1; }
echo "tests: $(tail -1 ${out}_tests.log)"
export SGV_AB=1
for rep in 1 2; do
  for v in 0 1; do
    SGV_MF_PAIR=$v timeout -k 10 300 python -u tools/ldpass_ab.py --tag "SGV_MF_PAIR=$v" \
        --shapes 64x15625,16x15625,8x15625,8x25000 --ncols 4,8 >> ${out}_ab.jsonl 2>> ${out}_ab.err || exit 1
  done
done
cat ${out}_ab.jsonl
for args in "--blocks 8" ""; do
  for v in 0 1; do
    SGV_MF_PAIR=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off \
        --read-bw 0 $args > ${out}_bench.tmp 2>> ${out}_bench.err || exit 1
    python -c "import json; d=json.load(open('${out}_bench.tmp')); print(json.dumps(dict(ab='SGV_MF_PAIR=$v', args='$args', value=round(d['value'],3), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4))))" | tee -a ${out}_bench.jsonl
  done
done
