#!/bin/bash
# Round 4: coupled band pieces -- the LD pass vs scipy, one band block over 2-3
# ranks bitwise vs one rank, the existing band / multi-rank suites.
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q \
    -k "coupled_pieces or band" --timeout 200 --timeout-method thread > gpurun_out/r04_cpl_parity.log 2>&1 \
    || { echo "coupled parity FAILED"; tail -40 gpurun_out/r04_cpl_parity.log; exit 1; }
echo "coupled parity: $(tail -1 gpurun_out/r04_cpl_parity.log)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v -k "single_band_block" \
    --timeout 280 --timeout-method thread > gpurun_out/r04_cpl_ranks.log 2>&1 \
    || { echo "band over ranks FAILED"; tail -60 gpurun_out/r04_cpl_ranks.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04_cpl_ranks.log | tail -5
