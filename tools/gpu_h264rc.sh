#!/bin/bash
# Default 1080p H.264 bench under CQP and CRF (no e2e, no 4K rows), a kernel trace of
# the CRF run, then the driver's default command (with the end-to-end session check).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-h264rc}
mkdir -p gpurun_out/$TAG
B="--steps 20 --warmup 5 --e2e-sessions 0 --extra-4k 0"
timeout -k 10 300 python bench.py $B --rc cqp > gpurun_out/$TAG/cqp.jsonl 2> gpurun_out/$TAG/cqp.err && tail -1 gpurun_out/$TAG/cqp.jsonl && \
timeout -k 10 300 python bench.py $B --rc crf > gpurun_out/$TAG/crf.jsonl 2> gpurun_out/$TAG/crf.err && tail -1 gpurun_out/$TAG/crf.jsonl && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" $B --rc crf > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log" 2>&1
rc=$?
cd "$GRAFT_REPO_ROOT"
DB=$(ls gpurun_out/$TAG/prof/*/run_results.db gpurun_out/$TAG/prof/run_results.db 2>/dev/null | head -1)
[ -n "$DB" ] && python tools/rocprof_summary.py "$DB" > gpurun_out/$TAG/kernels.md && head -24 gpurun_out/$TAG/kernels.md
[ $rc -eq 0 ] || exit $rc
if [ "${FULL:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/default.jsonl 2> gpurun_out/$TAG/default.err && tail -1 gpurun_out/$TAG/default.jsonl
fi
