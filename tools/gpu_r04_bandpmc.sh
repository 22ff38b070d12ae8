#!/bin/bash
# Round 4: why the band passes stop at 0.59 (8 columns) -- per-dispatch effective
# clock, MFMA busy and stall mix of the band pass (M = 1e6, bw = 1,000) next to the
# dense north-star blocks, and the band pass's HBM traffic (FETCH_SIZE, WRITE_SIZE).
# Summaries: python tools/clock_summary.py gpurun_out/bpmc_*; tools/pmc_summary.py
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
P="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
tools/gpu_steps.sh \
  "bpmc_band:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc $P -d $R/gpurun_out/bpmc_band -o pmc --output-format csv -- python3 $R/tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 8,16 --reps 3" \
  "bpmc_dense:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc $P -d $R/gpurun_out/bpmc_dense -o pmc --output-format csv -- python3 $R/tools/ldpass_ab.py --shapes 64x15625 --ncols 8 --reps 3" \
  "bpmc_fetch:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/bpmc_fetch -o pmc --output-format csv -- python3 $R/tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 8 --reps 3" \
  "bpmc_write:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/bpmc_write -o pmc --output-format csv -- python3 $R/tools/ldpass_band.py --M 1000000 --bw 1000 --ncols 8 --reps 3" || exit $?
# the band at VAMP level (bench --band: CSR -> coupled pieces -> the class seam),
# one GPU and two ranks sharing the card (the halo exchange over the host path)
tools/gpu_steps.sh \
  "bband1:420:timeout -k 10 400 python -u bench.py --band 1000000,1000 --steps 5 --warmup 2 --no-files > gpurun_out/bband1.json" \
  "bband2:420:timeout -k 10 400 python -u bench.py --band 1000000,1000 --steps 5 --warmup 2 --no-files --gpus 2 --share-device > gpurun_out/bband2.json"
