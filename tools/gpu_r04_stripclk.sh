#!/bin/bash
# Round 4: does the dense plan's clock follow its strip length?  The north
# star's 64 x 15,625 blocks at 8 columns with 3-, 5- and 8-panel strips
# (SGV_MFMA_STRIP): per-dispatch clock, MFMA busy, pass time.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
export SGV_AB=1
P="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
tools/gpu_steps.sh \
  "sc_3:240:cd /tmp && SGV_MFMA_STRIP=3 timeout -s KILL 220 rocprofv3 --pmc $P -d $R/gpurun_out/sc_3 -o pmc --output-format csv -- python3 $R/tools/ldpass_ab.py --shapes 64x15625,8x15625 --ncols 8 --reps 3" \
  "sc_5:240:cd /tmp && SGV_MFMA_STRIP=5 timeout -s KILL 220 rocprofv3 --pmc $P -d $R/gpurun_out/sc_5 -o pmc --output-format csv -- python3 $R/tools/ldpass_ab.py --shapes 64x15625,8x15625 --ncols 8 --reps 3" \
  "sc_8:240:cd /tmp && SGV_MFMA_STRIP=8 timeout -s KILL 220 rocprofv3 --pmc $P -d $R/gpurun_out/sc_8 -o pmc --output-format csv -- python3 $R/tools/ldpass_ab.py --shapes 64x15625,8x15625 --ncols 8 --reps 3"
