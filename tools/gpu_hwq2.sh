#!/bin/bash
# Driver-config bench: hardware queues x frames in flight.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for q in 4 8; do for f in 1 2; do
  GPU_MAX_HW_QUEUES=$q SK_CAPTURE_INFLIGHT=$f timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/hq_${q}_${f}_a.jsonl 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=$q SK_CAPTURE_INFLIGHT=$f timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/hq_${q}_${f}_a.jsonl 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=$q SK_CAPTURE_INFLIGHT=$f timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/hq_${q}_${f}_b.jsonl 2>&1 || exit 1
done; done
echo EXIT 0
