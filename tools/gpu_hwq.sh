#!/bin/bash
# Driver-config bench under different hardware-queue counts (HIP's GPU_MAX_HW_QUEUES).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/hwq_${q}_a.jsonl 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/hwq_${q}_b.jsonl 2>&1 || exit 1
done
echo EXIT 0
