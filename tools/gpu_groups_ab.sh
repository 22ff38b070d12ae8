export TMPDIR=/tmp SGV_AB=1
o=gpurun_out/grp3
for rep in 1 2 3; do
  for g in 1 4; do
    SGV_PASS_GROUPS=$g timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 > $o.$g.json 2>> $o.err || exit 1
    python3 -c "import json; d=json.load(open('$o.$g.json')); print(json.dumps(dict(groups=$g, value=round(d['value'],3), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4))))" | tee -a $o.jsonl
  done
done
