timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hevc_gpu.py tests/test_ratecontrol.py tests/test_gst_plugin.py > gpurun_out/r5h2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r5h2_tests.log; exit $rc
