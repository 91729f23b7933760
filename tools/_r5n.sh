A="--encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0"
bash tools/gpu_steps.sh \
 "tests r5n_tests tests/test_av1_gpu.py tests/test_gst_plugin.py tests/test_session_migration.py tests/test_rebalance.py tests/test_hevc_gpu.py tests/test_yuv_input.py tests/test_ratecontrol.py tests/test_h264_intra4x4.py tests/test_h264_gpu.py" \
 "pmc r5n_av1pmc $A" "prof r5n_av1prof $A" "driver r5n_driver"
