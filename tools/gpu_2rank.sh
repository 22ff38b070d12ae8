#!/bin/bash
# Two ranks on the one GPU (host exchange; RCCL refuses two ranks per device):
# the multi-rank bench path end to end (sharded blocks, replicated EM, ordered
# reductions), C2 and C3 shapes.  Timings are not a multi-GPU result.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "tworank_c2:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --share-device --steps 5 --warmup 2" \
  "tworank_c3:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --share-device --K 4 --steps 5 --warmup 2"
