#!/bin/bash
# Round 4: the band pass on a band whose every entry within bw is non-zero with
# genotype-LD-like values (ldpass_band.py --fill dense, M = 250,000, bw = 1,000)
# next to the synthetic windowed LD: pass time, then clock and MFMA busy.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
P="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
tools/gpu_steps.sh \
  "bdd_pass:500:timeout -k 10 480 python -u tools/ldpass_band.py --tag dense-fill --M 250000 --bw 1000 --fill dense --ncols 8,16 --reps 10 > gpurun_out/bdd_pass.jsonl" \
  "bdd_pmc:500:cd /tmp && timeout -s KILL 480 rocprofv3 --pmc $P -d $R/gpurun_out/bdd_pmc -o pmc --output-format csv -- python3 $R/tools/ldpass_band.py --M 250000 --bw 1000 --fill dense --ncols 8,16 --reps 3"
