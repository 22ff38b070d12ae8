set -o pipefail
cd $GRAFT_REPO_ROOT
SGV_FULL_GATE=1 SGV_GATE_LOG=gpurun_out/c3_ref_gate.log SGV_TEST_TIMES=gpurun_out/c3_ref_times.txt timeout -k 10 1100 python -u -m pytest tests/test_gpu_configs.py -x -q -p no:cacheprovider -k "c3_50_iterations" --timeout 1080 --timeout-method thread > gpurun_out/c3_ref_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/c3_ref_pytest.log; cat gpurun_out/c3_ref_times.txt; grep -v "oracle (reference algebra) iteration" gpurun_out/c3_ref_gate.log | tail -8
exit $rc
