#!/bin/bash
# Final-tree check: GPU suite, smoke(), default bench line.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
T=${1:-final}
tools/gpu_steps.sh \
  "gputests_$T:600:python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "smoke_$T:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench_$T:300:python bench.py"
