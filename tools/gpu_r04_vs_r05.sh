#!/bin/bash
# Same-box A/B of the north-star bench line: round 4's last tree (tools/r04snap:
# its bench.py and library, built from commit e8a64af) against this tree,
# alternating three times.  Extra arguments go to both bench lines.
#   bash tools/gpu_r04_vs_r05.sh TAG [bench args]
cd "$(dirname "$0")/.." || exit 2
o=gpurun_out/r04r05_${1:-ns}
shift
export TMPDIR=/tmp
for rep in 1 2 3; do
  for t in r04 r05; do
    B=bench.py; [ $t = r04 ] && B=tools/r04snap/bench.py
    timeout -k 10 300 python -u $B --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 "$@" > $o.$t.json 2>> $o.err || exit 1
    python3 -c "import json; d=json.load(open('$o.$t.json')); print(json.dumps(dict(tree='$t', value=round(d['value'],3), ms_pass=round(d['roofline']['avg_launch_ms'],4), frac=round(d['roofline']['frac'],4))))" | tee -a $o.jsonl
  done
done
