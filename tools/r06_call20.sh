set -o pipefail
cd $GRAFT_REPO_ROOT
export SGV_AB=1
SGV_MF16_TB=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -k "strips_vs_numpy or C5" --timeout 200 --timeout-method thread > gpurun_out/tb_parity.log 2>&1 || { tail -30 gpurun_out/tb_parity.log; exit 1; }
echo "parity TB=1: $(tail -1 gpurun_out/tb_parity.log)"
for rep in 1 2; do
  for v in 0 1; do
    SGV_MF16_TB=$v timeout -k 10 300 python -u tools/ldpass_ab.py --tag "TB=$v" --shapes 64x15625,8x15625 --ncols 16 >> gpurun_out/tb_ab.jsonl 2>> gpurun_out/tb_ab.err || exit 1
  done
done
python3 tools/ab_table.py gpurun_out/tb_ab.jsonl
for rep in 1 2; do
for v in 0 1; do
  for cfg in "c5:--K 8 --ridge 0.1 --lmmse-damp 1 --steps 3 --warmup 1" "c5conv:--K 8 --ridge 0.1 --lmmse-damp 1 --nsamp 20000 --steps 5 --warmup 2"; do
    name=${cfg%%:*}; args=${cfg#*:}
    SGV_MF16_TB=$v timeout -k 10 400 python -u bench.py --cpu-baseline off --read-bw 0 $args > gpurun_out/tbb_${name}_$v.json 2> gpurun_out/tbb_${name}_$v.err || { tail gpurun_out/tbb_${name}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/tbb_${name}_$v.json')); r=d['roofline']; c=d.get('compute_roofline') or {}; print(json.dumps(dict(ab='SGV_MF16_TB=$v', cfg='$name', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4), mfma_frac=c.get('frac'))))" | tee -a gpurun_out/tb_bench.jsonl
  done
done
done
