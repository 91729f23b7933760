#!/bin/bash
# GPU box: driver window with / without the copy-engine warm-up.
set -o pipefail
mkdir -p gpurun_out/win4
one() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --gpus 1 $BARGS > gpurun_out/win4/$name.jsonl 2>&1 || { tail -5 gpurun_out/win4/$name.jsonl; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/win4/$name.jsonl').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_encode_latency_ms'],d['p99_encode_latency_ms'])"
}
BARGS="--steps 20 --warmup 5"
one warm_a A=1 && one nowarm SK_COPY_WARMUP=0 && one warm_b A=1 && one warm_c A=1 && BARGS="--steps 200 --warmup 20" one warm_200 A=1
