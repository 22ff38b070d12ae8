#!/bin/bash
# The band bench's output files (one chromosome in coupled pieces, walks) from
# the tree's library and from tools/ablib/libsgvamp_hip_old.so, compared
# bitwise, then both timed alternately.  Swaps the library in the box's copy.
cd "$(dirname "$0")/.." || exit 2
o=gpurun_out/bbw
export TMPDIR=/tmp
cp sgvamp-py_amd/libsgvamp_hip.so gpurun_out/lib_new.so
run() {   # tag
  rm -rf $o.$1; mkdir -p $o.$1
  timeout -k 10 300 python -u bench.py --band 1000000,1000 --steps 3 --warmup 1 --cpu-baseline off \
      --read-bw 0 --out-dir $o.$1 > $o.$1.json 2>> $o.err || exit 1
}
run new
cp tools/ablib/libsgvamp_hip_old.so sgvamp-py_amd/libsgvamp_hip.so
run old
cp gpurun_out/lib_new.so sgvamp-py_amd/libsgvamp_hip.so
python3 tools/ab_bitwise_dirs.py $o.new $o.old || exit 1
for rep in 1 2; do
  for t in new old; do
    [ $t = old ] && cp tools/ablib/libsgvamp_hip_old.so sgvamp-py_amd/libsgvamp_hip.so
    timeout -k 10 300 python -u bench.py --band 1000000,1000 --steps 10 --warmup 2 --no-files \
        --cpu-baseline off --read-bw 0 > $o.t.json 2>> $o.err || exit 1
    cp gpurun_out/lib_new.so sgvamp-py_amd/libsgvamp_hip.so
    python3 -c "import json; d=json.load(open('$o.t.json')); print(json.dumps(dict(lib='$t', value=round(d['value'],2), ms_pass=round(d['roofline']['avg_launch_ms'],4))))" | tee -a $o.jsonl
  done
done
