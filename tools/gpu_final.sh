#!/bin/bash
# Driver command, kernel profile of the headline path, and 4K HEVC, on one MI355X.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-fin}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err && \
timeout -k 10 200 python bench.py --encoder hevc --width 3840 --height 2160 --sessions 1 --steps 30 --warmup 5 --e2e-sessions 0 > gpurun_out/${TAG}_hevc4k.jsonl 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_h264_s8" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 5 --e2e-sessions 0 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_h264_s8.log" 2>&1
echo EXIT $?
