#!/bin/bash
# AV1 on one MI355X: GPU==CPU parity tests, 4K / 1080p benches, kernel trace of the 4K run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-av1}
MODE=${2:-all}
mkdir -p gpurun_out/$TAG
if [ "$MODE" != "bench" ]; then
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_av1_entropy.py tests/test_av1_gpu.py \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
fi
timeout -k 10 200 python bench.py --encoder av1 --sessions 1 --width 3840 --height 2160 --steps 60 --warmup 10 --rc cbr --kbps 40000 --fps 120 \
    --e2e-sessions 0 --extra-4k 0 > gpurun_out/$TAG/bench_4k.jsonl 2>&1 && tail -1 gpurun_out/$TAG/bench_4k.jsonl && \
timeout -k 10 200 python bench.py --encoder av1 --sessions 8 --steps 30 --warmup 5 --mode fullframe \
    --e2e-sessions 0 --extra-4k 0 > gpurun_out/$TAG/bench_1080p.jsonl 2>&1 && tail -1 gpurun_out/$TAG/bench_1080p.jsonl && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --encoder av1 --sessions 1 --width 3840 --height 2160 --steps 20 --warmup 3 --rc cbr --kbps 40000 --fps 120 --e2e-sessions 0 --extra-4k 0 > "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log" 2>&1
rc=$?
cd "$GRAFT_REPO_ROOT"
DB=$(ls gpurun_out/$TAG/prof/*/run_results.db gpurun_out/$TAG/prof/run_results.db 2>/dev/null | head -1)
[ -n "$DB" ] && python tools/rocprof_summary.py "$DB" > gpurun_out/$TAG/kernels.md && head -30 gpurun_out/$TAG/kernels.md
exit $rc
