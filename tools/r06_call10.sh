set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ld_matvec or strips or pair or finalize or coupled" --timeout 120 --timeout-method thread > gpurun_out/ip_parity_default.log 2>&1 || { tail -30 gpurun_out/ip_parity_default.log; exit 1; }
tail -1 gpurun_out/ip_parity_default.log
export SGV_AB=1
SGV_MF_IP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ld_matvec or strips or pair or finalize or coupled" --timeout 120 --timeout-method thread > gpurun_out/ip_parity_1.log 2>&1 || { tail -30 gpurun_out/ip_parity_1.log; exit 1; }
echo "parity IP=1: $(tail -1 gpurun_out/ip_parity_1.log)"
bash tools/gpu_ab_multi.sh gpurun_out/ab_ip SGV_MF_IP "0 1" 64x15625,8x15625,8x25000 4,8 || exit $?
for rep in 1 2; do
for v in 0 1; do
  for cfg in "ns:" "ns8blk:--blocks 8 --block-size 15625 --K 4"; do
    name=${cfg%%:*}; args=${cfg#*:}
    SGV_MF_IP=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 $args > gpurun_out/ipb_${name}_$v.json 2> gpurun_out/ipb_${name}_$v.err || { tail gpurun_out/ipb_${name}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ipb_${name}_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_MF_IP=$v', cfg='$name', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/ip_bench.jsonl
  done
done
done
