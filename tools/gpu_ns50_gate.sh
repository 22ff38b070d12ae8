cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!
SGV_FULL_GATE=1 timeout -k 10 1120 python -u -m pytest tests/test_gpu_configs.py -x -s -q -k "north_star_50 and ${1:-4}" --timeout 1100 --timeout-method thread -p no:cacheprovider > gpurun_out/ns50_gate.log 2>&1
rc=$?
kill $HB
tail -12 gpurun_out/ns50_gate.log | cut -c1-600
exit $rc
