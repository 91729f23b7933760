#!/bin/bash
# GPU box: e2e session sweep with sharded clients, 1080p then 4K.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_e2e.py --sweep 8,12,15 --seconds 6 --warmup 5 --client-procs 4 \
    > gpurun_out/e2e2_1080p.jsonl 2> gpurun_out/e2e2_1080p.err || { tail -30 gpurun_out/e2e2_1080p.err; exit 1; }
cat gpurun_out/e2e2_1080p.jsonl | tail -1
timeout -k 10 300 python -u tools/bench_e2e.py --sweep 1,4,8 --width 3840 --height 2160 --seconds 6 --warmup 5 --client-procs 4 \
    > gpurun_out/e2e2_4k.jsonl 2> gpurun_out/e2e2_4k.err || { tail -30 gpurun_out/e2e2_4k.err; exit 1; }
cat gpurun_out/e2e2_4k.jsonl | tail -1
