#!/bin/bash
# A/B/C.. of an SGV_AB=1 switch: LD-pass parity under each non-default
# setting, the LD-pass microbenchmark (bitwise hashes) alternating the
# settings twice, and optionally a bench line per setting.
#   bash tools/gpu_ab_multi.sh <out-prefix> <VAR> "<v0 v1 ..>" <shapes> <ncols> [bench args...]
set -o pipefail
out=$1; var=$2; vals=$3; shapes=$4; ncols=$5
shift 5
export SGV_AB=1
for v in $vals; do
  env "$var=$v" timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
      -k "ld_matvec_vs_numpy and packed" --timeout 120 --timeout-method thread \
      > ${out}_parity_$v.log 2>&1 || { echo "parity $var=$v FAILED"; tail -30 ${out}_parity_$v.log; exit 1; }
  echo "parity $var=$v: $(tail -1 ${out}_parity_$v.log)"
done
for rep in 1 2; do
  for v in $vals; do
    env "$var=$v" timeout -k 10 300 python -u tools/ldpass_ab.py --tag "$var=$v" \
        --shapes $shapes --ncols $ncols >> ${out}_ab.jsonl 2>> ${out}_ab.err || exit 1
  done
done
cat ${out}_ab.jsonl
if [ $# -gt 0 ]; then
  for v in $vals; do
    env "$var=$v" timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off \
        --read-bw 0 "$@" > ${out}_bench_$v.tmp 2>> ${out}_bench.err || exit 1
    python -c "import json; d=json.load(open('${out}_bench_$v.tmp')); print(json.dumps(dict(ab='$var=$v', value=round(d['value'],3), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4), passes=d['ld_passes_per_step'])))"
  done
fi
