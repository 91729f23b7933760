bash tools/gpu_steps.sh \
 "tests r5k_tests tests/test_gst_plugin.py tests/test_session_migration.py tests/test_rebalance.py tests/test_hevc_gpu.py tests/test_yuv_input.py tests/test_ratecontrol.py tests/test_av1_gpu.py tests/test_h264_intra4x4.py tests/test_h264_gpu.py" \
 "profpy r5k_hk tools/key_latency.py --codec hevc --frames 24" \
 "py r5k_av1_4k tools/rc_trace.py --backend hip --codec av1 --width 3840 --height 2160 --fps 120 --kbps 40000 --frames 240 --pool 8 --json gpurun_out/r5k_av1_4k/av1_4k.json" \
 "py r5k_hevc_4k tools/rc_trace.py --backend hip --codec hevc --width 3840 --height 2160 --fps 60 --kbps 20000 --frames 240 --pool 8 --json gpurun_out/r5k_hevc_4k/hevc_4k.json" \
 "rate r5k_rate h264 hevc av1"
