set -o pipefail
bash tools/gpu.sh tests r5j_tests tests/test_hevc_gpu.py tests/test_yuv_input.py tests/test_gst_plugin.py tests/test_ratecontrol.py tests/test_av1_gpu.py tests/test_h264_intra4x4.py tests/test_h264_gpu.py tests/test_session_migration.py && \
bash tools/gpu.sh profpy r5j_hk tools/key_latency.py --codec hevc --frames 24 && \
bash tools/_r5g.sh
