#!/bin/bash
# Round 4 final-tree evidence (per-step limits, tools/gpu_steps.sh): GPU suite,
# smoke(), the default bench line, its kernel trace, the 8-rank share-device
# rehearsal line (exchange counters), distinct per-cohort LD at M = 1e6.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
T=${1:-r04final}
tools/gpu_steps.sh \
  "gputests_$T:900:python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "smoke_$T:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench_$T:300:python bench.py" \
  "trace_$T:400:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o bench --output-format csv -- python3 $R/bench.py" \
  "share8_$T:500:python bench.py --gpus 8 --share-device --steps 3 --warmup 1 --cpu-baseline off --read-bw 0" \
  "distinct4_$T:600:python bench.py --distinct-ld --K 4 --steps 3 --warmup 1 --cpu-baseline off --read-bw 0"
