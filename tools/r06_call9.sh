set -o pipefail
cd $GRAFT_REPO_ROOT
export SGV_AB=1
for w in 8 6 12 16; do
  SGV_WALK_LEN=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "band_vs_scipy or coupled_pieces" --timeout 120 --timeout-method thread > gpurun_out/walklen_parity_$w.log 2>&1 || { tail -20 gpurun_out/walklen_parity_$w.log; exit 1; }
  echo "parity W=$w: $(tail -1 gpurun_out/walklen_parity_$w.log)"
done
for rep in 1 2; do
  for w in 8 6 12 16; do
    SGV_WALK_LEN=$w timeout -k 10 300 python -u tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 4,8 --reps 5 --tag W=$w >> gpurun_out/walklen_ab.jsonl 2>> gpurun_out/walklen_ab.err || exit 1
  done
done
cat gpurun_out/walklen_ab.jsonl
for w in 8 6 12 16; do
  SGV_WALK_LEN=$w timeout -k 10 300 python -u bench.py --band 1000000,1000 --steps 10 --warmup 2 --no-files --cpu-baseline off --read-bw 0 > gpurun_out/walklen_bench_$w.json 2> gpurun_out/walklen_bench_$w.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/walklen_bench_$w.json')); r=d['roofline']; print(json.dumps(dict(W=$w, value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/walklen_bench.jsonl
done
