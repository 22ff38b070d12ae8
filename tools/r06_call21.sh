set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_multi.sh gpurun_out/ab_pair SGV_MF_PAIR "0 1" 8x15625,16x15625 5,8 --blocks 8 --block-size 15625 --K 4 || exit $?
export SGV_AB=1
for v in 0 1; do
  SGV_MF_PAIR=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 --blocks 8 --block-size 15625 --K 4 > gpurun_out/pairb2_$v.json 2> gpurun_out/pairb2_$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pairb2_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_MF_PAIR=$v', cfg='ns8blk', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))"
done
