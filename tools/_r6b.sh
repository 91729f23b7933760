# HEVC parity with the wave-per-unit binariser and the reworked 32x32 TU trial, then the 4K CRF kernel table
A="--encoder hevc --width 3840 --height 2160 --sessions 1 --fps 60 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0"
bash tools/gpu.sh tests r6b_t tests/test_hevc_gpu.py || exit $?
bash tools/gpu.sh prof r6b_p $A > /dev/null || exit $?
head -16 gpurun_out/r6b_p/kernels.md | cut -d'|' -f2-8
tail -1 gpurun_out/r6b_p/prof.log | cut -c1-300
