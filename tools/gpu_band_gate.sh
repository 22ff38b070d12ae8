#!/bin/bash
# The band path's full-size gate (tests/test_gpu_configs.py::test_band_full_size_vs_oracle,
# in the default suite too) with a heartbeat file.
cd $GRAFT_REPO_ROOT
( while true; do date >> gpurun_out/heartbeat.log; sleep 50; done ) &
HB=$!
SGV_FULL_GATE=1 timeout -k 10 1120 python -u -m pytest tests/test_gpu_configs.py -x -s -q -k "band_full_size" --timeout 1100 --timeout-method thread -p no:cacheprovider > gpurun_out/band_gate.log 2>&1
rc=$?
kill $HB
tail -8 gpurun_out/band_gate.log | cut -c1-600
exit $rc
