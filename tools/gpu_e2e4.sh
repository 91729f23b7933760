#!/bin/bash
# GPU box: why does the bench-embedded 8-session e2e check miss 60 fps when the standalone one sustains it?
set -o pipefail
mkdir -p gpurun_out/e2e4
timeout -k 10 200 python -u tools/bench_e2e.py --sweep 8 --seconds 4 --warmup 6 --client-procs 4 > gpurun_out/e2e4/standalone.jsonl 2>&1 || exit 1
tail -1 gpurun_out/e2e4/standalone.jsonl | cut -c1-400
timeout -k 10 200 python -u tools/bench_e2e.py --sweep 8 --seconds 8 --warmup 8 --client-procs 8 > gpurun_out/e2e4/standalone_long.jsonl 2>&1 || exit 1
tail -1 gpurun_out/e2e4/standalone_long.jsonl | cut -c1-400
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --e2e-seconds 8 > gpurun_out/e2e4/bench_long.jsonl 2>&1 || exit 1
tail -1 gpurun_out/e2e4/bench_long.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['e2e'])"
