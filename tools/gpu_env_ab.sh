#!/bin/bash
# A/B of an SGV_AB=1 environment switch of the in-tree library: LD-pass parity
# with the variant on, then tools/ldpass_ab.py alternating the values twice
# (ms per pass, SHA-256 of the products: equal SHA = bitwise the same).
#   bash tools/gpu_env_ab.sh <out-prefix> <VAR> "<v0 v1 ...>" <shapes> <ncols>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=$1; var=$2; vals=$3; shapes=$4; ncols=$5
last=${vals##* }
env SGV_AB=1 $var=$last timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "ld_matvec_vs_numpy and packed or mfma_strips" --timeout 120 --timeout-method thread \
    > ${out}_parity.log 2>&1 || { echo "parity FAILED"; tail -30 ${out}_parity.log; exit 1; }
echo "parity ($var=$last): $(tail -1 ${out}_parity.log)"
for rep in 1 2; do
  for v in $vals; do
    env SGV_AB=1 $var=$v timeout -k 10 300 python -u tools/ldpass_ab.py --tag $var=$v \
        --shapes $shapes --ncols $ncols >> ${out}_ab.jsonl 2>> ${out}_ab.err || exit 1
  done
done
cat ${out}_ab.jsonl
