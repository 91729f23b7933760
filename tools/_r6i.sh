# 1080p RD of all codecs (HEVC quadtree + rounding, H.264 automatic deblocking), HEVC and
# AV1 4K kernel tables of the current build
mkdir -p gpurun_out/r6i
timeout -k 10 600 python -u tools/rd_codecs.py --backend hip --width 1920 --height 1080 --frames 20 \
    --content motion,desktop --json gpurun_out/r6i/rd.json > gpurun_out/r6i/rd.md 2> gpurun_out/r6i/rd.err || { tail -5 gpurun_out/r6i/rd.err; exit 1; }
tail -6 gpurun_out/r6i/rd.md
bash tools/gpu.sh prof r6i_hevc --encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0 > /dev/null || exit $?
head -14 gpurun_out/r6i_hevc/kernels.md | cut -d'|' -f2-8
bash tools/gpu.sh prof r6i_av1 --encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 120 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0 > /dev/null || exit $?
head -14 gpurun_out/r6i_av1/kernels.md | cut -d'|' -f2-8
