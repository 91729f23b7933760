#!/bin/bash
# Default 1080p H.264 window of several checkouts (built in place), same box, in order.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-bisect}; shift
mkdir -p gpurun_out/$TAG
for d in "$@" .; do
  X="--steps 40 --warmup 5 --e2e-sessions 0"
  grep -q -- "--extra-4k" $d/bench.py && X="$X --extra-4k 0"
  grep -q -- '"--rc"' $d/bench.py && X="$X --rc cqp"
  n=$(basename $(cd $d && pwd))
  (cd $d && timeout -k 10 200 python bench.py $X) > gpurun_out/$TAG/$n.jsonl 2> gpurun_out/$TAG/$n.err || exit 1
  echo "$n $(tail -1 gpurun_out/$TAG/$n.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_encode_latency_ms"], d["p99_encode_latency_ms"])')"
done
