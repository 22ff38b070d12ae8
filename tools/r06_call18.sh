set -o pipefail
cd $GRAFT_REPO_ROOT
B=tools/ablib/libsgvamp_hip_base.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "band or coupled or coupling" --timeout 120 --timeout-method thread > gpurun_out/brow_parity.log 2>&1 || { tail -30 gpurun_out/brow_parity.log; exit 1; }
tail -1 gpurun_out/brow_parity.log
for rep in 1 2; do
  for lib in new base; do
    L=""; [ $lib = base ] && L="--lib $B"
    timeout -k 10 300 python -u tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 3,4,8 --tag "$lib" $L >> gpurun_out/brow_ab.jsonl 2>> gpurun_out/brow_ab.err || exit 1
  done
done
python3 tools/ab_table.py gpurun_out/brow_ab.jsonl
