#!/bin/bash
# Round 4: the clock the passes hold over a long run -- kernel traces of the
# north-star bench (100 steps, ~3.5 s of passes) right after the device set-up
# (whose generator kernels load the chip for seconds) and after 20 s of idle,
# and of the band bench (300 steps); per-dispatch durations over time
# (tools/drift_summary.py).
cd "$(dirname "$0")/.." || exit 2
R=$(pwd)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "drift_ns:300:cd /tmp && timeout -k 10 280 rocprofv3 --kernel-trace -d $R/gpurun_out/drift_ns -o t --output-format csv -- python3 $R/bench.py --steps 100 --warmup 3 --cpu-baseline off --read-bw 0" \
  "drift_nsp:300:cd /tmp && timeout -k 10 280 rocprofv3 --kernel-trace -d $R/gpurun_out/drift_nsp -o t --output-format csv -- python3 $R/bench.py --steps 100 --warmup 3 --cpu-baseline off --read-bw 0 --pause 20" \
  "drift_band:300:cd /tmp && timeout -k 10 280 rocprofv3 --kernel-trace -d $R/gpurun_out/drift_band -o t --output-format csv -- python3 $R/bench.py --band 1000000,1000 --steps 300 --warmup 3 --no-files --read-bw 0"
