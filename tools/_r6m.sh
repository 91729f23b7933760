# H.264 headline timeline: kernels + memory copies of the driver configuration (8 x 1080p capture sessions)
mkdir -p gpurun_out/r6m
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r6m/prof" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0 \
    > "$GRAFT_REPO_ROOT/gpurun_out/r6m/prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
tail -1 gpurun_out/r6m/prof.log | cut -c1-300
ls gpurun_out/r6m/prof/*/ gpurun_out/r6m/prof/ 2>/dev/null | head
