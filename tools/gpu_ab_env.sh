#!/bin/bash
# A/B of an SGV_AB=1 environment switch on the GPU box: LD-pass parity with
# the B setting, then the LD-pass microbenchmark (tools/ldpass_ab.py, bitwise
# hashes) and the north-star bench, alternating A and B processes.
#   bash tools/gpu_ab_env.sh <out-prefix> <VAR> <A> <B> [bench args...]
# AB_NCOLS / AB_SHAPES override the microbenchmark's column counts / block shapes.
set -o pipefail
out=$1; var=$2; va=$3; vb=$4
shift 4
export SGV_AB=1
env "$var=$vb" timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "ld_matvec_vs_numpy and packed" --timeout 120 --timeout-method thread \
    > ${out}_parity.log 2>&1 || { echo "parity FAILED"; tail -30 ${out}_parity.log; exit 1; }
tail -1 ${out}_parity.log
for v in $va $vb $va $vb; do
  env "$var=$v" timeout -k 10 300 python -u tools/ldpass_ab.py --tag "$var=$v" \
      --shapes ${AB_SHAPES:-64x15625,8x25000,8x15625} --ncols ${AB_NCOLS:-4,8} >> ${out}_ab.jsonl 2>> ${out}_ab.err || exit 1
done
for v in $va $vb $va $vb; do
  env "$var=$v" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off \
      --read-bw 0 "$@" > ${out}_bench_$v.tmp 2>> ${out}_bench.err || exit 1
  python -c "import json,sys; d=json.load(open('${out}_bench_$v.tmp')); print(json.dumps(dict(ab='$var=$v', value=round(d['value'],3), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4))))" >> ${out}_bench.jsonl
done
cat ${out}_ab.jsonl ${out}_bench.jsonl
