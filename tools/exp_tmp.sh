cd /root/repo
timeout -k 10 900 python tools/ldpass_bench.py --blocks 64 --block-size 15625 --formats packed --ncols 1,2,4,8 --reps 5 > gpurun_out/ns_1e6.log 2>&1
