#!/bin/bash
# Round 4: the band kernel (RAG instantiation, row MFMAs not deferred) holds
# 2.2-2.3 GHz on band LD while the dense NC = 8 kernel holds ~1.45 GHz at the
# same MFMA and HBM rates.  The band kernel on the dense north-star blocks
# (SGV_MF_RAG=1; bitwise the same products) and the dense kernel without the
# deferred row MFMAs (SGV_MF_DEFER=0): pass times, hashes and clocks.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
export SGV_AB=1
P="GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
tools/gpu_steps.sh \
  "rc_ab:600:for r in 1 2; do for v in base rag def0; do case \$v in base) E=;; rag) E=SGV_MF_RAG=1;; def0) E=SGV_MF_DEFER=0;; esac; env \$E timeout -k 10 200 python -u tools/ldpass_ab.py --tag \$v --shapes 64x15625,8x15625 --ncols 8 --reps 10 >> gpurun_out/rc_ab.jsonl || exit 1; done; done" \
  "rc_pmc_rag:300:cd /tmp && SGV_MF_RAG=1 timeout -s KILL 280 rocprofv3 --pmc $P -d $R/gpurun_out/rc_pmc_rag -o pmc --output-format csv -- python3 $R/tools/ldpass_ab.py --shapes 64x15625 --ncols 8 --reps 3" \
  "rc_pmc_base:300:cd /tmp && timeout -s KILL 280 rocprofv3 --pmc $P -d $R/gpurun_out/rc_pmc_base -o pmc --output-format csv -- python3 $R/tools/ldpass_ab.py --shapes 64x15625 --ncols 8 --reps 3"
