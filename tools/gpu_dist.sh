#!/bin/bash
# Distributed-band path on one MI355X: device-pointer upload + RCCL single-rank tests,
# then the --dist-bands bench at world 1 and the lockstep --gather bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-dist}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dist_banded.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --dist-bands --width 3840 --height 2160 --steps 30 --warmup 5 > gpurun_out/${TAG}_bench.jsonl 2>&1 && \
timeout -k 10 200 python bench.py --gather --path encoder --steps 30 --warmup 5 --e2e-sessions 0 >> gpurun_out/${TAG}_bench.jsonl 2>&1
rc=$?; cut -c1-400 gpurun_out/${TAG}_bench.jsonl; exit $rc
