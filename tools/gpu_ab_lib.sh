#!/bin/bash
# A/B of two builds of the library (e.g. tools/diaglib/libsgvamp_prev.so vs the
# in-tree one): LD-pass parity of the in-tree build, then tools/ldpass_ab.py
# alternating the two builds twice (ms per pass, SHA-256 of the products).
#   bash tools/gpu_ab_lib.sh <out-prefix> <libA> <libB> <shapes> <ncols>
set -o pipefail
out=$1; la=$2; lb=$3; shapes=$4; ncols=$5
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "ld_matvec_vs_numpy and packed" --timeout 120 --timeout-method thread \
    > ${out}_parity.log 2>&1 || { echo "parity FAILED"; tail -30 ${out}_parity.log; exit 1; }
echo "parity: $(tail -1 ${out}_parity.log)"
for rep in 1 2; do
  for l in $la $lb; do
    timeout -k 10 300 python -u tools/ldpass_ab.py --lib $l --tag $(basename $l) \
        --shapes $shapes --ncols $ncols >> ${out}_ab.jsonl 2>> ${out}_ab.err || exit 1
  done
done
cat ${out}_ab.jsonl
