#!/bin/bash
# Round 4: does the band pass's clock depend on how many stored band entries are
# non-zero?  The synthetic windowed LD (simulate.windowed_ld / oracle.banded_ld)
# fills ~9 % of its window at taps = 12 and ~54 % at taps = 42 (M = 250,000,
# bw = 1,000): pass times, then the per-dispatch clock / MFMA busy of each.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
P="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
tools/gpu_steps.sh \
  "bd_t12:300:timeout -k 10 280 python -u tools/ldpass_band.py --tag taps12 --M 250000 --bw 1000 --taps 12 --ncols 8,16 --reps 10 > gpurun_out/bd_t12.jsonl" \
  "bd_t42:300:timeout -k 10 280 python -u tools/ldpass_band.py --tag taps42 --M 250000 --bw 1000 --taps 42 --ncols 8,16 --reps 10 > gpurun_out/bd_t42.jsonl" \
  "bdp_t12:300:cd /tmp && timeout -s KILL 280 rocprofv3 --pmc $P -d $R/gpurun_out/bdp_t12 -o pmc --output-format csv -- python3 $R/tools/ldpass_band.py --M 250000 --bw 1000 --taps 12 --ncols 8,16 --reps 3" \
  "bdp_t42:300:cd /tmp && timeout -s KILL 280 rocprofv3 --pmc $P -d $R/gpurun_out/bdp_t42 -o pmc --output-format csv -- python3 $R/tools/ldpass_band.py --M 250000 --bw 1000 --taps 42 --ncols 8,16 --reps 3"
