#!/bin/bash
# GPU box: host-side trace (HIP API + roctx) of the driver command, to find the early all-session stalls.
set -o pipefail
mkdir -p gpurun_out/win5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace --marker-trace -d gpurun_out/win5/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/win5/prof.log 2>&1 || { tail -20 gpurun_out/win5/prof.log; exit 1; }
tail -1 gpurun_out/win5/prof.log
