#!/bin/bash
# pipelined CG: full GPU suite, then bench A/B (SGV_CG_PIPE=0 host-tested loop vs default)
cd /root/repo || exit 2
R=$(pwd)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "c2_host:200:SGV_CG_PIPE=0 python bench.py --cpu-baseline off" \
  "c2_pipe:200:python bench.py --cpu-baseline off" \
  "b1_host:200:SGV_CG_PIPE=0 python bench.py --blocks 1 --cpu-baseline off --steps 20" \
  "b1_pipe:200:python bench.py --blocks 1 --cpu-baseline off --steps 20" \
  "c3_host:200:SGV_CG_PIPE=0 python bench.py --K 4 --cpu-baseline off" \
  "c3_pipe:200:python bench.py --K 4 --cpu-baseline off" \
  "c2_pipe_trace:300:cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/c2tr -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --steps 5 --warmup 2"
