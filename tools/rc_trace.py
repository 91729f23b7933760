"""K10 rate-control traces: per-frame coded size and QP of a CBR / CRF session.

    python tools/rc_trace.py --backend hip --width 1920 --height 1080 --frames 600 \
        --content motion --mode cbr --kbps 8000 [--codec h264] [--json out.json]

Prints one JSON summary line (mean rate vs target, largest non-key frame in frame
budgets, frames above 1.5 budgets, guard re-encodes) and optionally writes the whole
trace. Sizes are the delivered packet bytes (stripe headers and parameter sets
included), so the summary is what a client receives, not the controller's own count.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def run(backend: str, width: int, height: int, frames: int, content: str, mode: str, kbps: int,
        codec: str = "h264", fps: float = 60.0, qp: int = 25, stripe_height: int = 64, pool: int = 0) -> dict:
    from selkies_gstreamer_amd.ops.native import H264Encoder
    from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
    src = SyntheticDesktop(width, height, kind=content)
    enc = H264Encoder(width, height, stripe_height=stripe_height, fullframe=codec != "h264", backend=backend,
                      codec=codec, qp=qp, fps=fps, rate_control=mode, bitrate_kbps=kbps)
    sizes, keys, qps, redo = [], [], [], []
    frames_pool = [src.frame(i) for i in range(pool)] if pool > 0 else None   # bench.py's cycling pool
    t0 = time.perf_counter()
    buf = []   # the controller's (fullness, vbv_size, budget, vbv_ms) before each frame, bits
    for t in range(frames):
        st = enc.rc_stats()
        buf.append((st.get("fullness", 0), st.get("vbv_size", 0), st.get("budget", 0), st.get("vbv_ms", 0)))
        pk = enc.encode(frames_pool[t % pool] if frames_pool else src.frame(t), t & 0xFFFF)
        sizes.append(sum(len(p.data) for p in pk))
        keys.append(any(p.key for p in pk))
        st = enc.rc_stats()
        qps.append(st.get("cur_qp", qp))
        redo.append(st.get("cur_redo", 0))
    wall = time.perf_counter() - t0
    st = enc.rc_stats()
    enc.close()
    budget = kbps * 1000 / fps / 8 if kbps else None
    mean_kbps = sum(sizes) * 8 * fps / len(sizes) / 1000
    non_key = [s for s, k in zip(sizes, keys) if not k]
    out = {"backend": backend, "codec": codec, "content": content, "mode": mode, "target_kbps": kbps,
           "width": width, "height": height, "fps": fps, "frames": frames, "mean_kbps": round(mean_kbps, 1),
           "kib_per_frame": round(sum(sizes) / len(sizes) / 1024, 2), "keyframes": sum(keys),
           "qp_min": min(qps), "qp_max": max(qps), "qp_mean": round(sum(qps) / len(qps), 2),
           "redos": st.get("redos", 0), "wall_s": round(wall, 2)}
    if budget:
        out["rate_ratio"] = round(mean_kbps / kbps, 4)
        out["max_nonkey_budgets"] = round(max(non_key) / budget, 3) if non_key else None
        out["nonkey_over_1p5"] = sum(1 for s in non_key if s > 1.5 * budget)
        out["nonkey_over_2p5"] = sum(1 for s in non_key if s > 2.5 * budget)
        # the per-frame cap (ratecontrol.h rc_frame_cap) from the controller's own buffer
        # before each frame: a 1.5-frame VBV (H.264 / HEVC), or AV1's 120 ms leaky bucket
        # (no overflow) with its 2.5-budget ceiling; 3 % over it is framing (stripe / NAL /
        # OBU headers the controller does not count)
        over = 0
        for s, k, (full, vbv, b, vms) in zip(sizes, keys, buf):
            cap = 4 * b if k else (min(vbv - full + b, 2.5 * b) if vms > 0 else vbv)
            over += int(not k and 8 * s > 1.03 * cap)
        out["nonkey_over_cap"] = over
        out["max_key_budgets"] = round(max((s for s, k in zip(sizes, keys) if k), default=0) / budget, 3)
    out["recoded_frames"] = sum(1 for r in redo if r)
    out["trace"] = {"bytes": sizes, "key": [int(k) for k in keys], "qp": qps, "redo": redo}
    return out


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--backend", default="cpu", choices=("cpu", "hip"))
    ap.add_argument("--codec", default="h264", choices=("h264", "hevc", "av1"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--content", default="motion", choices=("motion", "desktop", "noise"))
    ap.add_argument("--mode", default="cbr", choices=("cqp", "crf", "cbr"))
    ap.add_argument("--kbps", type=int, default=8000)
    ap.add_argument("--fps", type=float, default=60.0)
    ap.add_argument("--qp", type=int, default=25)
    ap.add_argument("--pool", type=int, default=0, help="cycle this many source frames (bench.py's pool)")
    ap.add_argument("--json", default="", help="write the full trace here")
    a = ap.parse_args()
    r = run(a.backend, a.width, a.height, a.frames, a.content, a.mode, a.kbps, a.codec, a.fps, a.qp, pool=a.pool)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(r, f)
    r.pop("trace")
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
