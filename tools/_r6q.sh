# HEVC parity after the decision tuning, then the 1080p RD table
bash tools/gpu.sh tests r6q_t tests/test_hevc_gpu.py || exit $?
mkdir -p gpurun_out/r6q
timeout -k 10 600 python -u tools/rd_codecs.py --backend hip --width 1920 --height 1080 --frames 20 \
    --content motion,desktop --json gpurun_out/r6q/rd.json > gpurun_out/r6q/rd.md 2> gpurun_out/r6q/rd.err || { tail -5 gpurun_out/r6q/rd.err; exit 1; }
tail -6 gpurun_out/r6q/rd.md
