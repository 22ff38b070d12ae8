#!/bin/bash
# Round-3 bench set on one GPU box: the north-star line with the CPU baselines,
# the distinct-per-cohort-LD workload (bench + kernel trace), C3 and the
# north star's N = 8 per-GPU share.  Usage: bash tools/gpu_round3_bench.sh <prefix>
set -o pipefail
out=${1:-gpurun_out/r03b}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {   # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python -u bench.py "$@" > ${out}_$name.json 2> ${out}_$name.err || {
    echo "$name FAILED"; tail -20 ${out}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('${out}_$name.json')); r=d['roofline']; print('$name', round(d['value'],3), 'it/s', round(r['avg_launch_ms'],4), 'ms/pass', round(r['frac'],4), 'passes/step', d['ld_passes_per_step'])"
}
run ns 600
run distinct 600 --blocks 8 --block-size 25000 --K 4 --distinct-ld --cpu-baseline off --read-bw 0
run c3 400 --blocks 8 --block-size 25000 --K 4 --cpu-baseline off --read-bw 0
run ns8blk 400 --blocks 8 --block-size 15625 --K 4 --cpu-baseline off --read-bw 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ${out}_prof_distinct -o run -- \
    python bench.py --blocks 8 --block-size 25000 --K 4 --distinct-ld --cpu-baseline off \
    --read-bw 0 --steps 5 > ${out}_prof_distinct.log 2>&1 || { echo "rocprof FAILED"; tail ${out}_prof_distinct.log; exit 1; }
find ${out}_prof_distinct -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} ${out}_distinct_kernel_stats.csv
head -12 ${out}_distinct_kernel_stats.csv
python -c "import json; d=json.load(open('${out}_ns.json')); print(json.dumps(d['cpu_baseline'], indent=1))"
