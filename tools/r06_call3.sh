set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_recipes.sh ab pkpair SGV_PK_PAIR "1 0" 64x15625,8x15625 5,8 || exit $?
export SGV_AB=1
for rep in 1 2; do
for v in 1 0; do
  for cfg in "ns:" "ns8blk:--blocks 8 --block-size 15625 --K 4"; do
    name=${cfg%%:*}; args=${cfg#*:}
    SGV_PK_PAIR=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 $args > gpurun_out/pkb_${name}_$v.json 2> gpurun_out/pkb_${name}_$v.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/pkb_${name}_$v.json')); r=d['roofline']; print(json.dumps(dict(ab='SGV_PK_PAIR=$v', cfg='$name', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/pkpair_bench.jsonl
  done
done
done
