# HEVC 8K kernel table (30 frames: the pool wraps into intra frames every 8)
bash tools/gpu.sh prof r6t_8k --encoder hevc --width 7680 --height 4320 --sessions 1 --fps 60 --steps 30 --warmup 6 --pool 8 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0 > /dev/null || exit $?
head -30 gpurun_out/r6t_8k/kernels.md | cut -d'|' -f2-8
