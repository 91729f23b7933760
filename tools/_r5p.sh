mkdir -p gpurun_out/r5p
# the Intra4x4 sub-slice test hung the last call: alone, serialised kernels with the HIP
# launch log (the last launch logged names the kernel), a short limit
AMD_SERIALIZE_KERNEL=3 AMD_LOG_LEVEL=3 SK_NO_GRAPHS=1 timeout -k 10 100 python -u -m pytest -x -v \
    tests/test_h264_intra4x4.py -k "subslice_keyframes_gpu" -m gpu > gpurun_out/r5p/sub.log 2>&1
rc=$?; echo "subslice rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r5p/sub.log | tail -5
[ $rc -eq 0 ] || exit $rc
A="--encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0"
bash tools/gpu_steps.sh \
 "tests r5p_tests tests/test_h264_intra4x4.py tests/test_h264_gpu.py tests/test_ratecontrol.py tests/test_av1_gpu.py" \
 "pmc r5p_av1pmc $A" "prof r5p_av1prof $A" "driver r5p_driver"
