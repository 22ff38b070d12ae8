#!/bin/bash
# Final-tree check: GPU suite, smoke(), default bench line, kernel trace of the same bench
# command (its pass times vs that run's own bench line: tools/trace_pass_summary.py).
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
T=${1:-final}
tools/gpu_steps.sh \
  "gputests_$T:600:python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "smoke_$T:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench_$T:300:python bench.py" \
  "trace_$T:400:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o bench --output-format csv -- python3 $R/bench.py"
