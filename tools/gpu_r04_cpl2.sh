#!/bin/bash
# Round 4: the LDS-staged coupling kernel (k_coupling_lds) -- bitwise test, then
# the band bench's kernel trace with each form (SGV_CPL_FORM=0/1).
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
export SGV_AB=1
tools/gpu_steps.sh \
  "cpl2_test:300:timeout -k 10 280 python -u -m pytest tests/test_gpu_parity.py -x -q -k 'coupling_forms or coupled_pieces or band_block_over' --timeout 200 --timeout-method thread" \
  "cpl2_t0:300:cd /tmp && SGV_CPL_FORM=0 timeout -k 10 280 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cpl2_t0 -o t --output-format csv -- python3 $R/bench.py --band 1000000,1000 --steps 20 --warmup 2 --no-files --read-bw 0" \
  "cpl2_t1:300:cd /tmp && SGV_CPL_FORM=1 timeout -k 10 280 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cpl2_t1 -o t --output-format csv -- python3 $R/bench.py --band 1000000,1000 --steps 20 --warmup 2 --no-files --read-bw 0"
