#!/bin/bash
# Whole GPU test tier on one MI355X, then (optional) the AV1 bench + kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-tier}
mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/$TAG/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/$TAG/pytest_gpu.log | tail -20; exit $rc; }
if [ "$2" = "av1" ]; then bash tools/gpu_av1.sh $TAG bench; fi
