# final round-5 kernel tables: H.264 headline config, HEVC 4K CRF, AV1 4K CBR
bash tools/gpu.sh prof r5f_h264 --steps 40 --warmup 5 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
bash tools/gpu.sh prof r5f_hevc --encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
bash tools/gpu.sh prof r5f_av1 --encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
for t in h264 hevc av1; do head -8 gpurun_out/r5f_$t/kernels.md | tail -3; done
