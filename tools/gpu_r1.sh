#!/bin/bash
# Round-1 GPU session: tests, bench, rocprof kernel trace of the bench.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "gputests:560:python -m pytest tests -m gpu -q -p no:cacheprovider -rf" \
  "bench:300:python bench.py" \
  "rocprof:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline off"
