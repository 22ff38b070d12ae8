#!/bin/bash
# Round 4: the register transposes checked against the LDS tile (probe), the
# counter-synchronised wave-pair kernel (SGV_MF_PAIR_MAP=2/3) vs the barrier one
# and the 4-wave kernel, then a kernel trace of the band passes.
set -o pipefail
timeout -k 10 60 ./tools/xpose_probe > gpurun_out/r04_xpose_probe.txt 2>&1 || exit 1
cat gpurun_out/r04_xpose_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mfma_pair_kernel_bitwise" \
    --timeout 200 --timeout-method thread > gpurun_out/r04_pairsync_tests.log 2>&1 || { tail -20 gpurun_out/r04_pairsync_tests.log; exit 1; }
export SGV_AB=1
for m in 2 3; do
  SGV_MF_PAIR=1 SGV_MF_PAIR_MAP=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      -k "ld_matvec_vs_numpy and packed" --timeout 120 --timeout-method thread > gpurun_out/r04_pairsync_parity_$m.log 2>&1 \
      || { echo "parity map $m FAILED"; tail -20 gpurun_out/r04_pairsync_parity_$m.log; exit 1; }
  echo "parity map $m: $(tail -1 gpurun_out/r04_pairsync_parity_$m.log)"
done
for rep in 1 2; do
  for v in "SGV_MF_PAIR=0" "SGV_MF_PAIR=1 SGV_MF_PAIR_MAP=0" "SGV_MF_PAIR=1 SGV_MF_PAIR_MAP=2" "SGV_MF_PAIR=1 SGV_MF_PAIR_MAP=3"; do
    env $v timeout -k 10 300 python -u tools/ldpass_ab.py --tag "$v" --shapes 64x15625,8x15625,8x25000 --ncols 4,8 >> gpurun_out/r04_pairsync_ab.jsonl 2>> gpurun_out/r04_pairsync_ab.err || exit 1
  done
done
python3 -c "
import json
for l in open('gpurun_out/r04_pairsync_ab.jsonl'):
    d = json.loads(l); print(d['tag'], d['shape'], d['ncol'], d['ms_per_pass'], d['sha'])"
unset SGV_AB
BAND_TRACE_ONLY=1 timeout -k 10 700 bash tools/gpu_r04_band.sh gpurun_out/r04_band
