#!/bin/bash
# Steady-state IDR cost on one MI355X: host timing, then a kernel trace of the same run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-idr}
mkdir -p gpurun_out
timeout -k 10 120 python tools/idr_latency.py 60 4 > gpurun_out/${TAG}_host.txt 2>&1 && cat gpurun_out/${TAG}_host.txt && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run -- python3 "$GRAFT_REPO_ROOT/tools/idr_latency.py" 60 4 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
echo EXIT $?
