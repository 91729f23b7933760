# AV1 GPU tests + the 4K AV1 bench profile (k_av1_tokens scratch / MV stack change)
mkdir -p gpurun_out/r5z
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_av1_gpu.py tests/test_av1_entropy.py tests/test_session_migration.py > gpurun_out/r5z/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5z/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu.sh prof r5z_av1prof --encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
head -14 gpurun_out/r5z_av1prof/kernels.md | tail -10; tail -1 gpurun_out/r5z_av1prof/prof.log | cut -c1-300
