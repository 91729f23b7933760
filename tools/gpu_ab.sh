#!/bin/bash
# A/B of the default 1080p H.264 encoder window: the tree in $AB (another checkout,
# built in place) against this one, alternating, same box. Then a 16-session e2e check.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}
AB=${AB:-ab_r2}
mkdir -p gpurun_out/$TAG
B="--steps 40 --warmup 5 --e2e-sessions 0 --extra-4k 0"
for i in 1 2; do
  (cd $AB && timeout -k 10 200 python bench.py ${B/--extra-4k 0/}) > gpurun_out/$TAG/old_$i.jsonl 2> gpurun_out/$TAG/old_$i.err || exit 1
  tail -1 gpurun_out/$TAG/old_$i.jsonl | cut -c 1-330
  timeout -k 10 200 python bench.py $B --rc cqp > gpurun_out/$TAG/new_$i.jsonl 2> gpurun_out/$TAG/new_$i.err || exit 1
  tail -1 gpurun_out/$TAG/new_$i.jsonl | cut -c 1-330
done
timeout -k 10 300 python tools/bench_e2e.py --sweep 16 --sessions-per-proc 8 --seconds 4 --client-procs 8 \
  --log-dir gpurun_out/$TAG/e2e_logs > gpurun_out/$TAG/e2e.jsonl 2>&1; tail -2 gpurun_out/$TAG/e2e.jsonl
