#!/bin/bash
# Round-3 check on one MI355X: GPU test tier, desktop-content bench (damage-driven upload)
# against motion content, and a kernel profile of one 4K HEVC session (SAO, quarter-pel,
# 35 intra modes). Usage: bash tools/gpu_r3.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r3}
mkdir -p gpurun_out/$TAG
bash tools/gpu_tier.sh $TAG && \
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --e2e-sessions 0 --extra-4k 0 --content desktop \
    > gpurun_out/$TAG/bench_desktop.jsonl 2>&1 && \
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --e2e-sessions 0 --extra-4k 0 --content motion \
    > gpurun_out/$TAG/bench_motion.jsonl 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_hevc4k" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --encoder hevc --width 3840 --height 2160 --sessions 1 --steps 40 \
    --warmup 5 --e2e-sessions 0 --extra-4k 0 > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof_hevc4k.log" 2>&1
echo EXIT $?
