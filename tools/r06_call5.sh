set -o pipefail
cd $GRAFT_REPO_ROOT
export SGV_AB=1
for v in 1 0; do
  SGV_STRIP_ORDER=$v timeout -k 10 200 python -u tools/strip_trace.py --lib tools/diaglib/libsgvamp_trace.so --shapes 8x15625,64x15625 --ncol 8 > gpurun_out/xcdtrace_$v.jsonl 2> gpurun_out/xcdtrace_$v.err || { tail gpurun_out/xcdtrace_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/xcdtrace_$v.jsonl'):
    d=json.loads(l); print('order=$v', d['shape'], 'span', d['span_us'], 'tail', d['tail_us'], 'util', d['slot_util'], 'xcd busy', [x['busy_us'] for x in d['per_xcd']], 'xcd end', [x['last_end'] for x in d['per_xcd']])"
done
bash tools/gpu_ab_multi.sh gpurun_out/ab_xorder SGV_STRIP_ORDER "1 0" 64x15625,8x15625,8x25000 4,8 || exit $?
for rep in 1 2; do
for v in 1 0; do
  for cfg in "ns:" "ns8blk:--blocks 8 --block-size 15625 --K 4"; do
    name=${cfg%%:*}; args=${cfg#*:}
    SGV_STRIP_ORDER=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 $args > gpurun_out/xob_${name}_$v.json 2> gpurun_out/xob_${name}_$v.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/xob_${name}_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_STRIP_ORDER=$v', cfg='$name', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/xorder_bench.jsonl
  done
done
done
