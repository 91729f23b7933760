mkdir -p gpurun_out/r4a
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_av1_gpu.py tests/test_av1_entropy.py tests/test_ratecontrol.py tests/test_h264_gpu.py tests/test_hevc_gpu.py > gpurun_out/r4a/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4a/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4a/pytest.log | tail; exit $rc; }
timeout -k 10 300 python -u tools/rc_trace.py --backend hip --codec av1 --width 3840 --height 2160 --frames 240 --fps 120 --kbps 40000 --json gpurun_out/r4a/av1_rc.json > gpurun_out/r4a/av1_rc.txt 2>&1 || exit 1
cut -c1-600 gpurun_out/r4a/av1_rc.txt
timeout -k 10 300 python -u bench.py --encoder av1 --width 3840 --height 2160 --sessions 1 --steps 120 --warmup 10 --e2e-sessions 0 --extra-4k 0 --rc cbr --kbps 40000 --fps 120 > gpurun_out/r4a/av1_bench.jsonl 2> gpurun_out/r4a/av1_bench.err || exit 1
tail -1 gpurun_out/r4a/av1_bench.jsonl | cut -c1-1200
