#!/bin/bash
# Experiment: default 1080p window with and without the K10 per-frame kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-rck}
mkdir -p gpurun_out/$TAG
B="--steps 40 --warmup 5 --e2e-sessions 0 --extra-4k 0 --rc cqp"
for i in 1 2; do
  timeout -k 10 200 python bench.py $B > gpurun_out/$TAG/with_$i.jsonl 2> gpurun_out/$TAG/with_$i.err || exit 1
  tail -1 gpurun_out/$TAG/with_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("with", d["value"], d["p50_encode_latency_ms"], d["p99_encode_latency_ms"])'
  SK_EXP_NO_RCK=1 timeout -k 10 200 python bench.py $B > gpurun_out/$TAG/without_$i.jsonl 2> gpurun_out/$TAG/without_$i.err || exit 1
  tail -1 gpurun_out/$TAG/without_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("without", d["value"], d["p50_encode_latency_ms"], d["p99_encode_latency_ms"])'
done
