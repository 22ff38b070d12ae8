#!/bin/bash
# Eight ranks on the one GPU (host exchange; RCCL refuses two ranks per device):
# the N = 8 partition of the north star (8 blocks per rank), the socket
# rendezvous with 8 ranks and the per-step EM exchange, end to end.  Timings
# are eight processes sharing one device; the per-iteration l2 must equal the
# one-rank run's (tools/gpu_2rank.sh's onerank_ns log).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "eightrank_ns:500:python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --share-device --steps 5 --warmup 2 --cpu-baseline off" \
  "onerank_ns8:300:python bench.py --steps 5 --warmup 2 --cpu-baseline off"
