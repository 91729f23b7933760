# K10 traces of the three codecs (1080p60 CBR 8 / 16 Mbit/s, motion / desktop, 600 frames each)
bash tools/gpu.sh rate r6l_rate h264 hevc av1 > /dev/null || exit $?
cat gpurun_out/r6l_rate/rate.md | head -40
