set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ld_matvec or strips or pair or finalize or coupled or band" --timeout 120 --timeout-method thread > gpurun_out/swdef_parity.log 2>&1 || { tail -30 gpurun_out/swdef_parity.log; exit 1; }
tail -1 gpurun_out/swdef_parity.log
for rep in 1 2; do
  timeout -k 10 300 python -u tools/ldpass_ab.py --tag "swdef" --shapes 64x15625,8x15625,8x25000 --ncols 3,4,8 >> gpurun_out/swdef_ab.jsonl 2>> gpurun_out/swdef_ab.err || exit 1
done
cat gpurun_out/swdef_ab.jsonl
