#!/bin/bash
# Round 4 last-tree evidence (per-step limits, tools/gpu_steps.sh): GPU suite,
# smoke(), the default bench line and its kernel trace, the driver's own
# multi-rank launch line rehearsed on one GPU (torch.distributed.run, 2 ranks,
# --share-device), the band bench.
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
T=${1:-fc}
tools/gpu_steps.sh \
  "gputests_$T:900:python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
  "smoke_$T:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench_$T:300:python bench.py" \
  "trace_$T:400:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o bench --output-format csv -- python3 $R/bench.py" \
  "torchrun2_$T:400:timeout -k 10 380 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --share-device --steps 3 --warmup 1 --cpu-baseline off --read-bw 0" \
  "band_$T:300:python bench.py --band 1000000,1000 --steps 10 --warmup 2 --no-files"
