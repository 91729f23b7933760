set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 300 python -u tools/rc_trace.py --backend hip --codec av1 --width 3840 --height 2160 --fps 120 --kbps 40000 --frames 240 --pool 8 --json gpurun_out/r5j/av1_4k.json > gpurun_out/r5j/av1.txt 2>&1 &&
timeout -k 10 300 python -u tools/rc_trace.py --backend hip --codec hevc --width 3840 --height 2160 --fps 60 --kbps 20000 --frames 240 --pool 8 --json gpurun_out/r5j/hevc_4k.json > gpurun_out/r5j/hevc.txt 2>&1 &&
cat gpurun_out/r5j/*.txt && bash tools/gpu.sh rate r5j_rate h264 hevc av1
