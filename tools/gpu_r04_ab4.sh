#!/bin/bash
# Round 4: register transposes after the bit_cast fix (probe, parity, pass A/B
# with product hashes, north-star bench per setting); the pair kernel's auto
# choice (3-4 columns) vs the 4-wave kernel on the 8-block share's bench line.
set -o pipefail
timeout -k 10 60 ./tools/xpose_probe > gpurun_out/r04_xpose_probe2.txt 2>&1 || exit 1
cat gpurun_out/r04_xpose_probe2.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mfma_pair_kernel_bitwise or mfma_strips_vs_numpy" \
    --timeout 200 --timeout-method thread > gpurun_out/r04_pair2_tests.log 2>&1 || { tail -20 gpurun_out/r04_pair2_tests.log; exit 1; }
echo "pair tests: $(tail -1 gpurun_out/r04_pair2_tests.log)"
timeout -k 10 900 bash tools/gpu_ab_multi.sh gpurun_out/r04_xp2 SGV_MF_XPOSE "0 1 2" 64x15625,8x15625 4,8 || exit 1
for rep in 1 2; do
  for v in 0 auto; do
    if [ $v = auto ]; then e=""; else e="SGV_AB=1 SGV_MF_PAIR=0"; fi
    env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off \
        --read-bw 0 --blocks 8 > gpurun_out/r04_pairauto_bench.tmp 2>> gpurun_out/r04_pairauto_bench.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r04_pairauto_bench.tmp')); print(json.dumps(dict(ab='pair=$v', value=round(d['value'],3), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4))))" | tee -a gpurun_out/r04_pairauto_bench.jsonl
  done
done
# band plans: deferred row MFMAs (SGV_BAND_DEF) and the 16-column prefetch depth (SGV_MF16_PD)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "band or coupled" \
    --timeout 200 --timeout-method thread > gpurun_out/r04_band2_parity.log 2>&1 || { tail -20 gpurun_out/r04_band2_parity.log; exit 1; }
echo "band parity: $(tail -1 gpurun_out/r04_band2_parity.log)"
for rep in 1 2; do
  for v in "SGV_BAND_DEF=0 SGV_MF16_PD=1" "SGV_BAND_DEF=1 SGV_MF16_PD=2"; do
    env SGV_AB=1 $v timeout -k 10 200 python -u tools/ldpass_band.py --tag "$v" \
        --M 1000000 --bw 1000 --ncols 8,16 --reps 10 >> gpurun_out/r04_band2_ab.jsonl 2>> gpurun_out/r04_band2_ab.err || exit 1
  done
done
python3 -c "
import json
for l in open('gpurun_out/r04_band2_ab.jsonl'):
    d = json.loads(l); print(d['tag'], d['ncol'], '%.4f ms' % d['ms_per_pass'], '%.3f' % d['frac_of_8TBs'], d['sha'])"
