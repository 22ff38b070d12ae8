set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_multi.sh gpurun_out/ab_lp SGV_MF_LP "-1 2 18 19 3" 64x15625,8x15625 4,8 || exit $?
export SGV_AB=1
for v in -1 2 18 19 3; do
  SGV_MF_LP=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 > gpurun_out/lpb_$v.json 2> gpurun_out/lpb_$v.err || { tail gpurun_out/lpb_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lpb_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_MF_LP=$v', cfg='ns', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/lp_bench.jsonl
done
