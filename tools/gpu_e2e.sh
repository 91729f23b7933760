#!/bin/bash
# GPU box: HIP server e2e test, then the end-to-end session sweep (<=15 server
# processes: the box allows 16 GPU processes per user).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_server_gpu.py \
    > gpurun_out/e2e_test.log 2>&1 || { tail -40 gpurun_out/e2e_test.log; exit 1; }
tail -5 gpurun_out/e2e_test.log
timeout -k 10 420 python -u tools/bench_e2e.py --sweep ${SWEEP:-1,4,8,12,15} --seconds 6 --warmup 4 \
    > gpurun_out/e2e_1080p.jsonl 2> gpurun_out/e2e_1080p.err || { tail -30 gpurun_out/e2e_1080p.err; exit 1; }
cat gpurun_out/e2e_1080p.jsonl
