bash tools/gpu_steps.sh \
 "tests r5r_tests tests/test_ratecontrol.py tests/test_av1_gpu.py" \
 "rate r5r_rate h264 hevc av1" \
 "py r5r_av1_4k tools/rc_trace.py --backend hip --codec av1 --width 3840 --height 2160 --fps 120 --kbps 40000 --frames 240 --pool 8 --json gpurun_out/r5r_av1_4k/av1_4k.json" \
 "py r5r_hevc_4k tools/rc_trace.py --backend hip --codec hevc --width 3840 --height 2160 --fps 60 --kbps 20000 --frames 240 --pool 8 --json gpurun_out/r5r_hevc_4k/hevc_4k.json"
