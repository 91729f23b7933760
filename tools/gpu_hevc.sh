#!/bin/bash
# HEVC on one MI355X: parity tests, then a short 4K / 1080p bench and kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-hv}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hevc_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --encoder hevc --sessions 1 --width 3840 --height 2160 --steps 30 --warmup 5 > gpurun_out/${TAG}_bench.jsonl 2>&1 && \
timeout -k 10 200 python bench.py --encoder hevc --sessions 8 --steps 30 --warmup 5 >> gpurun_out/${TAG}_bench.jsonl 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --encoder hevc --sessions 1 --width 3840 --height 2160 --steps 20 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
echo EXIT $?
SK_NATIVE_LIB=$GRAFT_REPO_ROOT/selkies_gstreamer_amd/_lib/libselkies_native_stamps.so timeout -k 10 120 python "$GRAFT_REPO_ROOT/tools/stamps_hevc_cabac.py" > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_stamps.txt" 2>&1
cat "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_stamps.txt"
