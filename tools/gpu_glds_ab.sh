#!/bin/bash
# LDS-DMA variant of the MFMA pass: parity, then A/B against the register
# version (alternating processes).  Usage (on the GPU box):
#   bash tools/gpu_glds_ab.sh <out-prefix> [variants...]
set -o pipefail
out=${1:-gpurun_out/glds}
shift
vars=${@:-0 2 0 2}
export SGV_AB=1
SGV_MF_GLDS=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "ld_matvec_vs_numpy and packed and not valu" --timeout 120 --timeout-method thread \
    > ${out}_parity.log 2>&1 || { echo "parity FAILED"; tail -30 ${out}_parity.log; exit 1; }
tail -2 ${out}_parity.log
for v in $vars; do
  SGV_MF_GLDS=$v timeout -k 10 300 python -u tools/ldpass_ab.py --tag glds$v \
      --shapes 64x15625,8x25000,8x15625 --ncols 4,8 >> ${out}_ab.jsonl 2>> ${out}_ab.err || exit 1
done
cat ${out}_ab.jsonl
