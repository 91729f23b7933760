#!/bin/bash
# GPU box: what makes early hipMemcpyAsync calls stall (7 ms, all sessions at once)?
set -o pipefail
mkdir -p gpurun_out/win3
one() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 $BARGS > gpurun_out/win3/$name.jsonl 2>&1 || return 1
  python -c "import json;d=json.loads(open('gpurun_out/win3/$name.jsonl').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_encode_latency_ms'],d['p99_encode_latency_ms'])"
}
one base A=1 && one nosdma HSA_ENABLE_SDMA=0 && BARGS="--pool 4" one pool4 A=1 && BARGS="--pool 32" one pool32 A=1 \
 && one base2 A=1 && one sdma_nocopy HSA_ENABLE_SDMA=1 HSA_ENABLE_PEER_SDMA=0
