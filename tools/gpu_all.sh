#!/bin/bash
# Full GPU tier: every @pytest.mark.gpu test, the driver smoke, and the 1-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.jsonl 2>&1
echo EXIT $?
