#!/bin/bash
# One 4K HEVC session (deblocking on) through the capture path + a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-hevc4k}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python bench.py --encoder hevc --sessions 1 --width 3840 --height 2160 --mode fullframe --steps 60 \
    --warmup 10 --e2e-sessions 0 --extra-4k 0 > gpurun_out/$TAG/bench_4k.jsonl 2>&1 && tail -1 gpurun_out/$TAG/bench_4k.jsonl && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --encoder hevc --sessions 1 --width 3840 --height 2160 --mode fullframe --steps 20 --warmup 3 --e2e-sessions 0 --extra-4k 0 > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log" 2>&1
rc=$?
cd "$GRAFT_REPO_ROOT"
DB=$(ls gpurun_out/$TAG/prof/*/run_results.db gpurun_out/$TAG/prof/run_results.db 2>/dev/null | head -1)
[ -n "$DB" ] && python tools/rocprof_summary.py "$DB" > gpurun_out/$TAG/kernels.md && head -16 gpurun_out/$TAG/kernels.md
exit $rc
