cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && tools/gpu_steps.sh \
 "abA:200:python tools/ab_bitwise.py --lib sgvamp-py_amd/libsgvamp_hip.so" \
 "abB:200:python tools/ab_bitwise.py --lib ab_lib/base.so" \
 "fintests:300:python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k \"ld_matvec or band or golden\"" \
 "trace_fin:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fin -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline off"
