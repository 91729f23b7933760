#!/bin/bash
# H.264 GPU correctness (bit-exact vs CPU) then bench + single-session kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r1}
timeout -k 10 600 python -m pytest tests/test_h264_gpu.py -x -q > gpurun_out/${TAG}_pytest_h264.log 2>&1 && \
timeout -k 10 240 python bench.py --steps 100 --warmup 10 > gpurun_out/${TAG}_bench_h264.jsonl 2>&1 && \
timeout -k 10 240 python bench.py --sessions 1 --steps 200 --warmup 10 >> gpurun_out/${TAG}_bench_h264.jsonl 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_h264_s1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --sessions 1 --steps 100 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_h264_s1.log" 2>&1
echo EXIT $?
