#!/bin/bash
# AV1 on one MI355X: GPU==CPU parity tests, then a kernel trace of a short 1080p / 4K run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-av1}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_av1_gpu.py \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
tail -25 gpurun_out/$TAG/pytest.log
exit $rc
