#!/bin/bash
# Intra wavefront iteration: stamps breakdown, H.264 parity tests, driver-config benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-it}
mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps_intra.py > gpurun_out/${TAG}_stamps.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_h264_gpu.py tests/test_capture_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.jsonl 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/${TAG}_bench.jsonl 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 20 >> gpurun_out/${TAG}_bench.jsonl 2>&1
echo EXIT $?
