# GPU parity of the rate control / HEVC / AV1 changes, 1080p RD, AV1 CBR traces, then the
# bench extras (4K and 8K, no e2e)
bash tools/gpu.sh tests r6d_t tests/test_ratecontrol.py tests/test_hevc_gpu.py tests/test_av1_gpu.py || exit $?
mkdir -p gpurun_out/r6d
timeout -k 10 600 python -u tools/rd_codecs.py --backend hip --width 1920 --height 1080 --frames 20 \
    --content motion,desktop --json gpurun_out/r6d/rd.json > gpurun_out/r6d/rd.md 2> gpurun_out/r6d/rd.err || { tail -5 gpurun_out/r6d/rd.err; exit 1; }
bash tools/gpu.sh rate r6d_rate av1 > /dev/null || exit $?
tail -8 gpurun_out/r6d_rate/rate.md
bash tools/gpu.sh bench r6d_b --steps 20 --warmup 5 --e2e-sessions 0 --e2e-av1 none > /dev/null || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6d_b/bench.jsonl").read().strip().splitlines()[-1])
print(d["value"], d["p50_encode_latency_ms"])
for k in ("hevc_4k", "hevc_4k_cbr", "av1_4k", "hevc_8k", "av1_8k"):
    v = d.get(k, {})
    if "error" in v or "fps" not in v:
        print(k, v); continue
    print(k, v["fps"], v["p50_encode_latency_ms"], v["p99_encode_latency_ms"], v["keyframe"]["latency_ms"], v["kib_per_frame"], v["paced"]["p99_encode_latency_ms"])
PY
