set -o pipefail
cd $GRAFT_REPO_ROOT
export SGV_AB=1
SGV_MF_SW=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ld_matvec or strips or finalize or coupled" --timeout 120 --timeout-method thread > gpurun_out/sw_parity_1.log 2>&1 || { tail -30 gpurun_out/sw_parity_1.log; exit 1; }
echo "parity SW=1: $(tail -1 gpurun_out/sw_parity_1.log)"
bash tools/gpu_ab_multi.sh gpurun_out/ab_sw SGV_MF_SW "0 1" 64x15625,8x15625,8x25000 4,8 || exit $?
for rep in 1 2; do
for v in 0 1; do
  for cfg in "ns:" "ns8blk:--blocks 8 --block-size 15625 --K 4"; do
    name=${cfg%%:*}; args=${cfg#*:}
    SGV_MF_SW=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 $args > gpurun_out/swb_${name}_$v.json 2> gpurun_out/swb_${name}_$v.err || { tail gpurun_out/swb_${name}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/swb_${name}_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_MF_SW=$v', cfg='$name', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/sw_bench.jsonl
  done
done
done
