set -o pipefail
cd $GRAFT_REPO_ROOT
export SGV_AB=1
for rep in 1 2; do
  for v in 0 1; do
    SGV_MF_PAIR=$v timeout -k 10 300 python -u tools/ldpass_ab.py --tag "SGV_MF_PAIR=$v" --shapes 8x25000,32x15625 --ncols 5,8 >> gpurun_out/c3pair_ab.jsonl 2>> gpurun_out/c3pair_ab.err || exit 1
  done
done
python3 tools/ab_table.py gpurun_out/c3pair_ab.jsonl
for rep in 1 2; do
  for v in 0 1; do
    SGV_MF_PAIR=$v timeout -k 10 300 python -u bench.py --blocks 8 --block-size 25000 --K 4 --cpu-baseline off --read-bw 0 > gpurun_out/c3pairb_$v.json 2> gpurun_out/c3pairb_$v.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/c3pairb_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_MF_PAIR=$v', cfg='c3', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/c3pair_bench.jsonl
  done
done
