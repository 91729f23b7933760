#!/bin/bash
# Where the end-to-end session ceiling comes from: 48 and 64 sessions (session hosts of 8)
# with CPU sampling per server process / thread, clients and GPU busy.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-collapse}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python tools/bench_e2e.py --sweep 48,64 --sessions-per-proc 8 --seconds 5 --warmup 6 --client-procs 8 \
  --sample-cpu --log-dir gpurun_out/$TAG/logs > gpurun_out/$TAG/e2e.jsonl 2>&1; rc=$?
tail -3 gpurun_out/$TAG/e2e.jsonl | cut -c 1-1500
exit $rc
