# H.264 / rate-control parity after the k_rc_qp change, then the headline (no extras) twice
bash tools/gpu.sh tests r6r_t tests/test_ratecontrol.py tests/test_h264_gpu.py || exit $?
bash tools/gpu.sh bench r6r_b1 --steps 200 --warmup 20 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0 || exit $?
bash tools/gpu.sh prof r6r_p --steps 200 --warmup 20 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0 > /dev/null || exit $?
grep -E "k_rc_qp|k_code_inter" gpurun_out/r6r_p/kernels.md | cut -d'|' -f2-8
