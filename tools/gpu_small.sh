#!/bin/bash
# Per-rank view of the 8-GPU strong-scaling step: C2's per-GPU share (one LD
# block of 25,000) on one GPU, with and without a one-rank RCCL communicator,
# plus a kernel trace for tools/step_timeline.py; and C3 (K=4) on the new MFMA pass.
cd /root/repo || exit 2
R=$(pwd)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "b1:200:python bench.py --blocks 1 --cpu-baseline off --steps 20" \
  "b1_rccl:200:python bench.py --blocks 1 --cpu-baseline off --steps 20 --exchange rccl" \
  "b1_trace:300:cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/b1tr -o run --output-format csv -- python3 $R/bench.py --blocks 1 --cpu-baseline off --steps 10" \
  "c3:200:python bench.py --K 4 --cpu-baseline off"
