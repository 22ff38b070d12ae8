set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_recipes.sh ab mf16 SGV_MF16 "2 1 8 9" 64x15625,8x15625 12,16 --K 8 --ridge 0.1 --lmmse-damp 1 --nsamp 20000 || exit $?
timeout -k 10 200 python -u tools/strip_trace.py --lib tools/diaglib/libsgvamp_trace.so --shapes 8x15625,64x15625 --ncol 8 > gpurun_out/striptrace_r06.jsonl 2> gpurun_out/striptrace_r06.err || exit $?
cat gpurun_out/striptrace_r06.jsonl
bash tools/gpu_recipes.sh trace ns8 --blocks 8 --block-size 15625 --K 4
