#!/bin/bash
# Round 4: band plans' MFMA strips over 256-column chunks (default) vs the
# round-3 512-column strips (SGV_BAND_CW=512): band parity vs scipy (both), pass
# times at M = 1e6, bw = 1,000 and M = 200k, bw = 2,000, 8 and 16 columns, and
# the coupled-piece / band-over-ranks tests on the default.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "band or coupled" \
    --timeout 200 --timeout-method thread > gpurun_out/r04_b256_parity.log 2>&1 || { echo "band default parity FAILED"; tail -30 gpurun_out/r04_b256_parity.log; exit 1; }
echo "band default parity: $(tail -1 gpurun_out/r04_b256_parity.log)"
SGV_AB=1 SGV_BAND_CW=256 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "band or coupled" \
    --timeout 200 --timeout-method thread > gpurun_out/r04_b512_parity.log 2>&1 || { echo "band256 (A/B) parity FAILED"; tail -30 gpurun_out/r04_b512_parity.log; exit 1; }
echo "band256 (A/B) parity: $(tail -1 gpurun_out/r04_b512_parity.log)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -q -k "single_band_block" \
    --timeout 280 --timeout-method thread > gpurun_out/r04_b256_ranks.log 2>&1 || { echo "band ranks FAILED"; tail -30 gpurun_out/r04_b256_ranks.log; exit 1; }
echo "band over ranks: $(tail -1 gpurun_out/r04_b256_ranks.log)"
for rep in 1 2; do
  for v in 512 256; do
    for cfg in "1000000 1000" "200000 2000"; do
      set -- $cfg
      env SGV_AB=1 SGV_BAND_CW=$v timeout -k 10 200 python -u tools/ldpass_band.py --tag "cw=$v" \
          --M $1 --bw $2 --ncols 4,8,16 --reps 10 >> gpurun_out/r04_b256_ab.jsonl 2>> gpurun_out/r04_b256_ab.err || exit 1
    done
  done
done
python3 -c "
import json
for l in open('gpurun_out/r04_b256_ab.jsonl'):
    d = json.loads(l); print(d['tag'], d['M'], d['bw'], d['ncol'], '%.4f ms' % d['ms_per_pass'], '%.3f' % d['frac_of_8TBs'], d['sha'])"
