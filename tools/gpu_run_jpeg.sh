#!/bin/bash
# GPU check of the JPEG path: tests, benches, kernel profile (outputs under gpurun_out/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r1}
timeout -k 10 600 python -m pytest tests/test_jpeg_gpu.py -x -q > gpurun_out/${TAG}_pytest_jpeg.log 2>&1 && \
timeout -k 10 180 python bench.py --encoder jpeg --steps 100 --warmup 10 > gpurun_out/${TAG}_bench_jpeg.jsonl 2>&1 && \
timeout -k 10 180 python bench.py --encoder jpeg --sessions 1 --steps 200 --warmup 10 >> gpurun_out/${TAG}_bench_jpeg.jsonl 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_jpeg" -o jpeg -- python3 "$GRAFT_REPO_ROOT/bench.py" --encoder jpeg --sessions 1 --steps 50 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_jpeg.log" 2>&1
echo EXIT $?
