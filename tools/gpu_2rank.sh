#!/bin/bash
# Two ranks on the one GPU (host exchange; RCCL refuses two ranks per device):
# the multi-rank bench path end to end (sharded blocks, ordered reductions, the
# size-chosen EM mode: one exchange per EM step at the north star, replicated at
# C2).  Timings are not a multi-GPU result; the per-iteration l2 must equal the
# one-rank run's.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "tworank_ns:400:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --share-device --steps 5 --warmup 2 --cpu-baseline off" \
  "onerank_ns:300:python bench.py --steps 5 --warmup 2 --cpu-baseline off" \
  "tworank_c2:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --share-device --blocks 8 --block-size 25000 --K 1 --steps 5 --warmup 2"
