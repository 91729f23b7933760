#!/bin/bash
# GPU box: driver window after moving uploads off the kernel stream.
set -o pipefail
mkdir -p gpurun_out/win8
one() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --gpus 1 $BARGS > gpurun_out/win8/$name.jsonl 2>&1 || { tail -5 gpurun_out/win8/$name.jsonl; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/win8/$name.jsonl').read().strip().splitlines()[-1]);print('$name',d['value'],d['p50_encode_latency_ms'],d['p99_encode_latency_ms'])"
}
BARGS="--steps 20 --warmup 5"
one w_a A=1 && one w_b A=1 && one w_c A=1 && one nowarm SK_COPY_WARMUP=0 \
 && BARGS="--steps 200 --warmup 20" one w_200 A=1 \
 && BARGS="--steps 20 --warmup 5 --encoder jpeg" one jpeg A=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_h264_gpu.py tests/test_jpeg_gpu.py > gpurun_out/win8/pytest.log 2>&1; tail -2 gpurun_out/win8/pytest.log
