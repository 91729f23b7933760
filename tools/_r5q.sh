A="--encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0"
bash tools/gpu_steps.sh \
 "tests r5q_tests tests/test_av1_gpu.py tests/test_ratecontrol.py tests/test_hevc_gpu.py" \
 "prof r5q_av1prof $A" "driver r5q_driver" \
 "py r5q_av1_4k tools/rc_trace.py --backend hip --codec av1 --width 3840 --height 2160 --fps 120 --kbps 40000 --frames 240 --pool 8 --json gpurun_out/r5q_av1_4k/av1_4k.json" \
 "py r5q_hevc_4k tools/rc_trace.py --backend hip --codec hevc --width 3840 --height 2160 --fps 60 --kbps 20000 --frames 240 --pool 8 --json gpurun_out/r5q_hevc_4k/hevc_4k.json" \
 "rate r5q_rate h264 hevc av1"
