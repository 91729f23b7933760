#!/bin/bash
# GPU box: where does the driver window's fixed cost come from? steps x warmup matrix + kernel trace of the driver command.
set -o pipefail
mkdir -p gpurun_out/win
for sw in "20 5" "20 50" "20 200" "40 5" "80 5" "200 20"; do
  set -- $sw
  timeout -k 10 120 python bench.py --gpus 1 --steps $1 --warmup $2 > gpurun_out/win/b_$1_$2.jsonl 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/win/b_$1_$2.jsonl').read().strip().splitlines()[-1]);print('$1 $2',d['value'],d['p50_encode_latency_ms'],d['p99_encode_latency_ms'])"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/win/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/win/prof.log 2>&1 || { tail -20 gpurun_out/win/prof.log; exit 1; }
tail -1 gpurun_out/win/prof.log
