# k_av1_cdf: 16 context partitions per tile (this tree) vs 32 (tools/ab/libcdf_p32.so)
for v in "frame --frames 12 --kbps 40000" "frame --frames 30 --kbps 40000" "frame" "frame --frames 6 --qp 30"; do
  tag=r5y_$(echo $v | tr -d ' -')
  bash tools/gpu.sh profpy $tag tools/cdf_micro.py --libs $PWD/tools/ab/libcdf_new.so,$PWD/tools/ab/libcdf_p32.so --variant $v > /dev/null || exit $?
  python - $tag "$v" <<'PY'
import sqlite3, glob, sys, statistics
tag = sys.argv[1]
db = (glob.glob(f"gpurun_out/{tag}/prof/*/run_results.db") + glob.glob(f"gpurun_out/{tag}/prof/run_results.db"))[0]
rows = [r for r in sqlite3.connect(db).execute("select name, duration, grid_x from kernels order by start") if "k_av1_cdf" in r[0]]
m = [r[1] / 1e3 for r in rows[-10:]]
o, n = statistics.median(m[:5]), statistics.median(m[5:])
print(f"| {sys.argv[2]} | {o:.0f} | {n:.0f} | {100 * (n - o) / o:+.1f} % |")
PY
done
