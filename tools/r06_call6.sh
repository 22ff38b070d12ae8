set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ld_matvec or strips or pair or finalize or coupled" --timeout 120 --timeout-method thread > gpurun_out/split_parity.log 2>&1 || { tail -30 gpurun_out/split_parity.log; exit 1; }
tail -2 gpurun_out/split_parity.log
bash tools/gpu_ab_multi.sh gpurun_out/ab_split SGV_STRIP_SPLIT "1 0" 8x15625,16x15625,8x25000 4,8,16 || exit $?
export SGV_AB=1
for rep in 1 2; do
for v in 1 0; do
  for cfg in "ns8blk:--blocks 8 --block-size 15625 --K 4" "c5s8:--blocks 8 --block-size 15625 --K 8 --ridge 0.1 --lmmse-damp 1 --nsamp 20000"; do
    name=${cfg%%:*}; args=${cfg#*:}
    SGV_STRIP_SPLIT=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 $args > gpurun_out/spb_${name}_$v.json 2> gpurun_out/spb_${name}_$v.err || { tail gpurun_out/spb_${name}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/spb_${name}_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_STRIP_SPLIT=$v', cfg='$name', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/split_bench.jsonl
  done
done
done
for v in 1 0; do
  SGV_STRIP_SPLIT=$v timeout -k 10 200 python -u tools/strip_trace.py --lib tools/diaglib/libsgvamp_trace.so --shapes 8x15625 --ncol 8 > gpurun_out/splittrace_$v.jsonl 2> gpurun_out/splittrace_$v.err || { tail gpurun_out/splittrace_$v.err; exit 1; }
  cut -c1-100 gpurun_out/splittrace_$v.jsonl; python -c "
import json; d=json.loads(open('gpurun_out/splittrace_$v.jsonl').readline()); print('split=$v span', d['span_us'], 'tail', d['tail_us'], 'util', d['slot_util'], 'strips', d['strips'])"
done
