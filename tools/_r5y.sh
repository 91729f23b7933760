# AV1 GPU tests, the k_av1_cdf A/B (round-4 kernel vs this tree) and the 4K AV1 bench profile
mkdir -p gpurun_out/r5y
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_av1_gpu.py tests/test_av1_entropy.py > gpurun_out/r5y/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5y/tests.log; [ $rc -eq 0 ] || exit $rc
for v in "frame --frames 12 --kbps 40000" "frame --frames 30 --kbps 40000" "frame" "frame --frames 6 --qp 30" "hot"; do
  tag=r5y_$(echo $v | tr -d ' -')
  bash tools/gpu.sh profpy $tag tools/cdf_micro.py --libs $PWD/tools/ab/libcdf_old.so,$PWD/tools/ab/libcdf_new.so --variant $v > /dev/null || exit $?
  python - $tag "$v" <<'PY' | tee -a gpurun_out/r5y/ab.txt
import sqlite3, glob, sys, statistics
tag = sys.argv[1]
db = (glob.glob(f"gpurun_out/{tag}/prof/*/run_results.db") + glob.glob(f"gpurun_out/{tag}/prof/run_results.db"))[0]
rows = [r for r in sqlite3.connect(db).execute("select name, duration, grid_x from kernels order by start") if "k_av1_cdf" in r[0]]
m = [r[1] / 1e3 for r in rows[-10:]]
o, n = statistics.median(m[:5]), statistics.median(m[5:])
print(f"| {sys.argv[2]} | {o:.0f} | {n:.0f} | {100 * (n - o) / o:+.1f} % |")
PY
done
bash tools/gpu.sh prof r5y_av1prof --encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 60 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 > /dev/null || exit $?
head -12 gpurun_out/r5y_av1prof/kernels.md; tail -1 gpurun_out/r5y_av1prof/prof.log | cut -c1-400
timeout -k 10 200 python -u tools/key_latency.py --codec av1 --frames 24 > gpurun_out/r5y/key.txt 2>&1 || exit $?
tail -2 gpurun_out/r5y/key.txt
