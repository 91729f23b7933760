#!/bin/bash
# H.264 parity tests + driver-config bench + kernel trace (one MI355X).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_h264_gpu.py tests/test_capture_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.jsonl 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 >> gpurun_out/${TAG}_bench.jsonl 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
echo EXIT $?
