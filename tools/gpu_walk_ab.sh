#!/bin/bash
# Band walks (band_walk.hip) vs the strip kernels on band plans: band parity
# tests (walks on by default), then the band pass microbenchmark and the band
# bench line alternating SGV_BAND_WALK=1 / 0 (SGV_AB=1), then a kernel trace.
#   bash tools/gpu_walk_ab.sh TAG
cd "$(dirname "$0")/.." || exit 2
T=${1:-w}
o=gpurun_out/walk_$T
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q \
    -p no:cacheprovider -k "band or coupled or coupling or finalize_forms" --timeout 300 \
    --timeout-method thread > $o.parity.log 2>&1 || { echo "parity FAILED"; tail -40 $o.parity.log; exit 1; }
tail -2 $o.parity.log
export SGV_AB=1
for rep in 1 2; do
  for v in 8 0; do
    SGV_BAND_WALK=$v timeout -k 10 300 python -u tools/ldpass_band.py --M 1000000 --bw 1000 \
        --ncols 3,4,8 --tag walk=$v >> $o.ab.jsonl 2>> $o.ab.err || exit 1
  done
done
cat $o.ab.jsonl
for rep in 1 2; do
  for v in 4 0; do
    SGV_BAND_WALK=$v timeout -k 10 300 python -u bench.py --band 1000000,1000 --steps 10 --warmup 2 \
        --no-files --read-bw 0 > $o.bench_$v.json 2>> $o.bench.err || exit 1
    python -c "import json; d=json.load(open('$o.bench_$v.json')); print(json.dumps(dict(walk=$v, value=round(d['value'],2), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4), cg=d['cg_iters_per_step'][-1])))" | tee -a $o.bench.jsonl
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_walk_$T \
    -o band --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --band 1000000,1000 --steps 10 \
    --warmup 2 --no-files --read-bw 0 > $GRAFT_REPO_ROOT/$o.trace.log 2>&1
echo "trace rc=$?"
