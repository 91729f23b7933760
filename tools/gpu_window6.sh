#!/bin/bash
# GPU box: are the early copy stalls triggered by munmap (glibc returning memory)?
set -o pipefail
mkdir -p gpurun_out/win6
one() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/win6/$name.jsonl 2>&1 || { tail -5 gpurun_out/win6/$name.jsonl; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/win6/$name.jsonl').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_encode_latency_ms'],d['p99_encode_latency_ms'])"
}
one base A=1 && one nommap MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=4294967296 MALLOC_TOP_PAD_=268435456 \
 && one base2 A=1 && one nommap2 MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=4294967296 MALLOC_TOP_PAD_=268435456 \
 && one nosdma HSA_ENABLE_SDMA=0
