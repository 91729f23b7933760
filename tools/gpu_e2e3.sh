#!/bin/bash
# GPU box: does HW-queue oversubscription (15 processes x 4 queues) cause the 1080p drop at 12+ sessions?
set -o pipefail
mkdir -p gpurun_out
for q in 1 2; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u tools/bench_e2e.py --sweep 12,15 --seconds 6 --warmup 5 --client-procs 4 \
    > gpurun_out/e2e3_q$q.jsonl 2> gpurun_out/e2e3_q$q.err || { tail -30 gpurun_out/e2e3_q$q.err; exit 1; }
tail -1 gpurun_out/e2e3_q$q.jsonl
done
