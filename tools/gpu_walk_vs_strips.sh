#!/bin/bash
# Band walks vs band strips on one box: the pass microbenchmark at 3, 4, 8 and
# 16 columns and the band bench line, alternating SGV_BAND_WALK=8 / 0 twice.
#   bash tools/gpu_walk_vs_strips.sh TAG
cd "$(dirname "$0")/.." || exit 2
T=${1:-ws}
o=gpurun_out/wvs_$T
mkdir -p gpurun_out
export TMPDIR=/tmp SGV_AB=1
for rep in 1 2; do
  for v in 8 0; do
    SGV_BAND_WALK=$v timeout -k 10 300 python -u tools/ldpass_band.py --M 1000000 --bw 1000 \
        --ncols 3,4,8,16 --tag walk=$v >> $o.ab.jsonl 2>> $o.err || exit 1
  done
done
python3 tools/ab_table.py $o.ab.jsonl
for rep in 1 2; do
  for v in 8 0; do
    SGV_BAND_WALK=$v timeout -k 10 300 python -u bench.py --band 1000000,1000 --steps 10 --warmup 2 \
        --no-files --read-bw 0 --cpu-baseline off > $o.bench_$v.json 2>> $o.err || exit 1
    python3 -c "import json; d=json.load(open('$o.bench_$v.json')); print(json.dumps(dict(walk=$v, value=round(d['value'],2), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4))))" | tee -a $o.bench.jsonl
  done
done
