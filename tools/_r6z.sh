# live-move cost at 1080p H.264 / 4K HEVC / 4K AV1 (old encoder + staging released off the capture thread)
bash tools/gpu.sh tests r6z_t tests/test_rebalance.py tests/test_capture_pipeline.py || exit $?
mkdir -p gpurun_out/r6z
timeout -k 10 300 python -u tools/move_stall.py > gpurun_out/r6z/move.jsonl 2> gpurun_out/r6z/move.err || { tail -20 gpurun_out/r6z/move.err; exit 1; }
cat gpurun_out/r6z/move.jsonl
