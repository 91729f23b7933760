#!/bin/bash
# H.264 on one MI355X: GPU==CPU parity tests, the driver bench, steady-state IDR cost,
# and a kernel trace of the driver bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-h264}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_h264_subpel.py tests/test_h264_gpu.py tests/test_overlay.py tests/test_session_migration.py tests/test_parallel_banded.py tests/test_dist_banded.py tests/test_h264_intra4x4.py -m gpu > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --e2e-sessions 0 > gpurun_out/$TAG/bench.jsonl 2>&1 || exit 1
tail -1 gpurun_out/$TAG/bench.jsonl | cut -c1-240
timeout -k 10 120 python tools/idr_latency.py 60 4 > gpurun_out/$TAG/idr.txt 2>&1 || exit 1
cat gpurun_out/$TAG/idr.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run -- python3 tools/idr_latency.py 60 4 > gpurun_out/$TAG/prof.log 2>&1 || exit 1
echo prof ok
