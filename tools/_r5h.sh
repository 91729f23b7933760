# HEVC GPU tests + 4K CRF kernel profile (SAO row decisions / packed offsets)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hevc_gpu.py tests/test_ratecontrol.py > gpurun_out/r5h_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r5h_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu.sh prof r5h_hevc2 --encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
head -14 gpurun_out/r5h_hevc2/kernels.md | tail -10; grep -E "k_hevc_sao" gpurun_out/r5h_hevc2/kernels.md; tail -1 gpurun_out/r5h_hevc2/prof.log | grep -o '"value": [0-9.]*'
