#!/bin/bash
# Effective shader clock and stall mix of the LD passes (round 3): GRBM_GUI_ACTIVE
# with SQ wave-cycle buckets per dispatch, for the north-star blocks at NC = 2
# (VALU pass), 4, 8 (MFMA 4x4x4), 12/16 (MFMA 16x16x4), against a streaming-read
# probe of the same traversal (tools/read_layout) and the MFMA issue-rate probe.
# Summaries: python tools/clock_summary.py gpurun_out/clk_*
#   tools/gpu_clock_evidence.sh   (build the probes first: see tools/README.md)
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
P="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
tools/gpu_steps.sh \
  "clk_passes:240:cd /tmp && timeout -s KILL 220 rocprofv3 --pmc $P -d $R/gpurun_out/clk_passes -o pmc --output-format csv -- python3 $R/tools/ldpass_ab.py --shapes 64x15625 --ncols 2,4,8,12,16 --reps 3" \
  "clk_read:120:cd /tmp && timeout -s KILL 100 rocprofv3 --pmc $P -d $R/gpurun_out/clk_read -o pmc --output-format csv -- $R/tools/read_layout" \
  "clk_mfma:120:cd /tmp && timeout -s KILL 100 rocprofv3 --pmc $P -d $R/gpurun_out/clk_mfma -o pmc --output-format csv -- $R/tools/mfma_probe"
