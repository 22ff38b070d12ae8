set -o pipefail
cd $GRAFT_REPO_ROOT
B=tools/ablib/libsgvamp_hip_base.so
N=sgvamp-py_amd/libsgvamp_hip.so
cp $N gpurun_out/lib_new.so
for rep in 1 2; do
  for lib in new base; do
    L=""; [ $lib = base ] && L="--lib $B"
    timeout -k 10 300 python -u tools/ldpass_ab.py --tag "$lib" --shapes 8x25000,64x15625 --ncols 5,6,7,8 $L >> gpurun_out/c3reg_ab.jsonl 2>> gpurun_out/c3reg_ab.err || exit 1
  done
done
python3 tools/ab_table.py gpurun_out/c3reg_ab.jsonl
for rep in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then cp $B $N; else cp gpurun_out/lib_new.so $N; fi
    timeout -k 10 300 python -u bench.py --blocks 8 --block-size 25000 --K 4 --cpu-baseline off --read-bw 0 > gpurun_out/c3reg_$lib.json 2> gpurun_out/c3reg_$lib.err || { tail gpurun_out/c3reg_$lib.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/c3reg_$lib.json')); r=d['roofline']; print(json.dumps(dict(lib='$lib', cfg='c3', value=round(d['value'],3), ms_pass=round(r['avg_launch_ms'],4), frac=round(r['frac'],4))))" | tee -a gpurun_out/c3reg_bench.jsonl
  done
done
cp gpurun_out/lib_new.so $N
rm -f gpurun_out/lib_new.so
