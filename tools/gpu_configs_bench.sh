#!/bin/bash
# Every BASELINE.json configuration's bench line on one GPU box (final tree):
# the north star (with its CPU baselines), C2, C3, C4, C5, distinct per-cohort
# LD and the north star's N = 8 per-GPU share.
#   bash tools/gpu_configs_bench.sh <prefix>
set -o pipefail
out=${1:-gpurun_out/cfg}
run() {   # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python -u bench.py "$@" > ${out}_$name.json 2> ${out}_$name.err || {
    echo "$name FAILED"; tail -20 ${out}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('${out}_$name.json')); r=d['roofline']; print(json.dumps(dict(config='$name', value=round(d['value'],3), ms_per_step=round(d['ms_per_step'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4), passes=round(d['ld_passes_per_step'],2), stream=r.get('box_stream_GBs'))))"
}
run ns 600
run c2 400 --blocks 8 --block-size 25000 --K 1 --cpu-baseline off --read-bw 0
run c3 400 --blocks 8 --block-size 25000 --K 4 --cpu-baseline off --read-bw 0
run c4 400 --K 1 --cpu-baseline off --read-bw 0
run c5 400 --K 8 --ridge 0.1 --lmmse-damp 1 --steps 3 --warmup 1 --cpu-baseline off --read-bw 0
run distinct 600 --blocks 8 --block-size 25000 --K 4 --distinct-ld --cpu-baseline off --read-bw 0
run ns8blk 400 --blocks 8 --block-size 15625 --K 4 --cpu-baseline off --read-bw 0
