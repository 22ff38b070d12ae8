set -o pipefail
cd $GRAFT_REPO_ROOT
export SGV_AB=1
SGV_MF_RC=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ld_matvec or strips or finalize or coupled" --timeout 120 --timeout-method thread > gpurun_out/rc_parity.log 2>&1 || { tail -30 gpurun_out/rc_parity.log; exit 1; }
echo "parity RC=1: $(tail -1 gpurun_out/rc_parity.log)"
bash tools/gpu_ab_multi.sh gpurun_out/ab_rc SGV_MF_RC "0 1" 64x15625,16x15625,8x25000 4,8 || exit $?
for rep in 1 2; do
for v in 0 1; do
  for cfg in "ns:" "c3:--blocks 8 --block-size 25000 --K 4"; do
    name=${cfg%%:*}; args=${cfg#*:}
    SGV_MF_RC=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 $args > gpurun_out/rcb_${name}_$v.json 2> gpurun_out/rcb_${name}_$v.err || { tail gpurun_out/rcb_${name}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/rcb_${name}_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_MF_RC=$v', cfg='$name', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/rc_bench.jsonl
  done
done
done
