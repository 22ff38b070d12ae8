set -o pipefail
cd $GRAFT_REPO_ROOT
SGV_TRACE_RAW=gpurun_out/strips_raw timeout -k 10 200 python -u tools/strip_trace.py --lib tools/diaglib/libsgvamp_trace.so --shapes 8x15625,64x15625 --ncol 8 > gpurun_out/striptrace2.jsonl 2> gpurun_out/striptrace2.err || { tail gpurun_out/striptrace2.err; exit 1; }
cat gpurun_out/striptrace2.jsonl
