set -o pipefail
bash tools/gpu.sh tests r5i_tests tests/test_yuv_input.py tests/test_gst_plugin.py tests/test_ratecontrol.py && bash tools/_r5g.sh
