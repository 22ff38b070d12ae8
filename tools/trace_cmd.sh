set -e
cd /root/repo
timeout -k 10 400 python -m pytest tests/test_gpu_multirank.py -q -m gpu -k rehearsal > gpurun_out/rehearsal.log 2>&1
timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --exchange rccl > gpurun_out/bench_rccl.log 2>&1
timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --exchange host > gpurun_out/bench_host.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /root/repo/gpurun_out/trace -o run -- python3 /root/repo/bench.py --cpu-baseline off --steps 8 > /root/repo/gpurun_out/bench_trace.log 2>&1
