#!/bin/bash
# GPU box: quarter-pel parity, then the driver bench and a kernel table.
set -o pipefail
mkdir -p gpurun_out/sp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_h264_subpel.py tests/test_h264_gpu.py tests/test_overlay.py -m gpu > gpurun_out/sp/pytest.log 2>&1 || { tail -40 gpurun_out/sp/pytest.log; exit 1; }
tail -2 gpurun_out/sp/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --e2e-sessions 0 > gpurun_out/sp/bench.jsonl 2>&1 || exit 1
tail -1 gpurun_out/sp/bench.jsonl | cut -c1-240
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sp/prof -o run -- python3 bench.py --gpus 1 --steps 100 --warmup 10 --e2e-sessions 0 > gpurun_out/sp/prof.log 2>&1 || exit 1
echo prof ok
