#!/bin/bash
# rocm-smi power, clocks and temperature every 2 s during a 400-step north-star bench
# (gpurun_out/pw_smi.log, pw_bench.log).
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 400 --warmup 3 --cpu-baseline off --no-files > gpurun_out/pw_bench.log 2>&1 &
BP=$!
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  sleep 2
  timeout -k 5 20 rocm-smi --showpower --showclocks --showtemp >> gpurun_out/pw_smi.log 2>&1
  echo "---- t=$((i*2))" >> gpurun_out/pw_smi.log
done
wait $BP
echo "bench rc=$?"
