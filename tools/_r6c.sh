# 1080p RD of the three codecs against round 5's table, then the bench extras (no e2e)
mkdir -p gpurun_out/r6c
timeout -k 10 600 python -u tools/rd_codecs.py --backend hip --width 1920 --height 1080 --frames 20 \
    --content motion,desktop --vs profiles/r5_rd_codecs_1080p.md --json gpurun_out/r6c/rd.json \
    > gpurun_out/r6c/rd.md 2> gpurun_out/r6c/rd.err || { tail -5 gpurun_out/r6c/rd.err; exit 1; }
tail -12 gpurun_out/r6c/rd.md
bash tools/gpu.sh bench r6c_b --steps 20 --warmup 5 --e2e-sessions 0 --e2e-av1 none > /dev/null || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6c_b/bench.jsonl").read().strip().splitlines()[-1])
print(d["value"], d["p50_encode_latency_ms"])
for k in ("hevc_4k", "hevc_4k_cbr", "av1_4k"):
    v = d[k]
    print(k, v["fps"], v["p50_encode_latency_ms"], v["p99_encode_latency_ms"], v["keyframe"]["latency_ms"], v["kib_per_frame"], v["paced"]["p99_encode_latency_ms"])
PY
