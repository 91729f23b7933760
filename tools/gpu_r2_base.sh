#!/bin/bash
# Round-2 baseline on one MI355X: GPU test tier, smoke, driver-config bench, long bench, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.jsonl 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 20 >> gpurun_out/${TAG}_bench.jsonl 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
echo EXIT $?
