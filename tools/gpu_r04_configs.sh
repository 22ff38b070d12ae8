#!/bin/bash
# Round 4 last tree: one bench line per BASELINE.json configuration on one GPU
# (C2, C3 at M = 200k; C4, C5 and the north star at M = 1e6), same box.
cd "$(dirname "$0")/.." || exit 2
B="--cpu-baseline off --read-bw 0"
tools/gpu_steps.sh \
  "cfg:900:for c in C2 C3 C4 C5 NS; do case \$c in C2) F='--K 1 --blocks 8 --block-size 25000';; C3) F='--K 4 --blocks 8 --block-size 25000';; C4) F='--K 1';; C5) F='--K 8 --ridge 0.1 --lmmse-damp 1';; NS) F='';; esac; timeout -k 10 170 python bench.py \$F $B | grep '^{' | sed \"s/^{/{\\\"cfg\\\": \\\"\$c\\\", /\" >> gpurun_out/cfg.jsonl || exit 1; done"
