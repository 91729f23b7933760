# 8K extras only (HEVC CRF, HEVC CBR 40 Mbit/s, AV1 CBR)
mkdir -p gpurun_out/r6v
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --e2e-sessions 0 --e2e-av1 none --extra-4k 0 --extra-8k 1 \
    > gpurun_out/r6v/bench.jsonl 2> gpurun_out/r6v/bench.err || { tail -20 gpurun_out/r6v/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6v/bench.jsonl").read().strip().splitlines()[-1])
for k in ("hevc_8k", "hevc_8k_cbr", "av1_8k"):
    e = d[k]
    print(k, e["fps"], e["p99_encode_latency_ms"], e["paced"]["p50_encode_latency_ms"], e["paced"]["p99_encode_latency_ms"],
          e["keyframe"]["latency_ms"], e["kib_per_frame"], e["realtime_at_source_rate"])
PY
