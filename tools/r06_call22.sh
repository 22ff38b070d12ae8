set -o pipefail
cd $GRAFT_REPO_ROOT
B=tools/ablib/libsgvamp_hip_base.so
N=sgvamp-py_amd/libsgvamp_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q -k "ld_matvec or strips or pair or finalize or coupled or sharded or rehearsal or multirank" --timeout 200 --timeout-method thread > gpurun_out/p58_parity.log 2>&1 || { tail -30 gpurun_out/p58_parity.log; exit 1; }
tail -1 gpurun_out/p58_parity.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -k "sharded" --timeout 300 --timeout-method thread > gpurun_out/p58_sharded.log 2>&1 || { tail -30 gpurun_out/p58_sharded.log; exit 1; }
tail -1 gpurun_out/p58_sharded.log
for rep in 1 2; do
  for lib in new base; do
    L=""; [ $lib = base ] && L="--lib $B"
    timeout -k 10 300 python -u tools/ldpass_ab.py --tag "$lib" --shapes 8x15625,16x15625,4x15625,2x25000 --ncols 5,8 $L >> gpurun_out/p58_ab.jsonl 2>> gpurun_out/p58_ab.err || exit 1
  done
done
python3 tools/ab_table.py gpurun_out/p58_ab.jsonl
cp $N gpurun_out/lib_new.so
for rep in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then cp $B $N; else cp gpurun_out/lib_new.so $N; fi
    for cfg in "ns8blk:--blocks 8 --block-size 15625 --K 4" "ns:"; do
      name=${cfg%%:*}; args=${cfg#*:}
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off --read-bw 0 $args > gpurun_out/p58b_${name}_$lib.json 2> gpurun_out/p58b_${name}_$lib.err || { tail gpurun_out/p58b_${name}_$lib.err; cp gpurun_out/lib_new.so $N; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/p58b_${name}_$lib.json')); r=d['roofline']; print(json.dumps(dict(lib='$lib', cfg='$name', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/p58_bench.jsonl
    done
  done
done
cp gpurun_out/lib_new.so $N
rm -f gpurun_out/lib_new.so
