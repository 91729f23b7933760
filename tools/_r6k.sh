# capture-path HEVC / AV1 CBR parity (no H.264 deblocking on their front end), AV1 4K table, bench extras
bash tools/gpu.sh tests r6k_t tests/test_jpeg_gpu.py tests/test_av1_gpu.py || exit $?
bash tools/gpu.sh prof r6k_av1 --encoder av1 --width 3840 --height 2160 --sessions 1 --fps 120 --rc cbr --kbps 40000 --steps 120 --warmup 10 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 0 > /dev/null || exit $?
head -18 gpurun_out/r6k_av1/kernels.md | cut -d'|' -f2-8
bash tools/gpu.sh bench r6k_b --steps 20 --warmup 5 --e2e-sessions 0 --e2e-av1 none > /dev/null || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6k_b/bench.jsonl").read().strip().splitlines()[-1])
print(d["value"], d["p50_encode_latency_ms"])
for k in ("hevc_4k", "hevc_4k_cbr", "av1_4k", "hevc_8k", "av1_8k"):
    v = d.get(k, {})
    print(k, v.get("fps"), v.get("p50_encode_latency_ms"), v.get("p99_encode_latency_ms"), v.get("keyframe", {}).get("latency_ms"), v.get("kib_per_frame"), v.get("paced", {}).get("p99_encode_latency_ms"))
PY
