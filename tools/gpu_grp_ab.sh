#!/bin/bash
# one-off: block-grouped two-stream MFMA pass A/B
cd "$(dirname "$0")/.." 2>/dev/null || true
export SGV_AB=1
o=gpurun_out/grp
mkdir -p gpurun_out
timeout -k 10 600 bash tools/gpu_ab_multi.sh $o SGV_PASS_GROUPS "1 2 4 8" 64x15625,8x15625 4,8 || exit 1
for rep in 1 2; do
 for g in 1 4; do
  SGV_PASS_GROUPS=$g timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 > $o.ns_$g.json 2>>$o.bench.err || exit 1
  python -c "import json; d=json.load(open('$o.ns_$g.json')); print(json.dumps(dict(cfg='ns',g=$g, value=round(d['value'],3), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4))))" | tee -a $o.bench.jsonl
 done
 for g in 1 2; do
  SGV_PASS_GROUPS=$g timeout -k 10 200 python -u bench.py --blocks 8 --steps 20 --warmup 3 --cpu-baseline off --read-bw 0 > $o.sh_$g.json 2>>$o.bench.err || exit 1
  python -c "import json; d=json.load(open('$o.sh_$g.json')); print(json.dumps(dict(cfg='share8',g=$g, value=round(d['value'],3), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4))))" | tee -a $o.bench.jsonl
 done
done
