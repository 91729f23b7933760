"""Cost of a live GPU move of a running capture session (csrc/runtime/capture.cpp
CaptureSession::move_to): the capture thread's stall between two frames (`move_stall_ms`),
the wall time of the move_to call (the target encoder is built off the capture thread),
and the capture->packet latency of the frames around the move. One GPU on the box, so the
session moves GPU 0 -> GPU 0 (a fresh encoder and a device-to-device state copy; across GPUs
the copy runs over xGMI peer access instead).

    python tools/move_stall.py            # H.264 1080p, HEVC 4K, AV1 4K; one JSON line each
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import pixelflux  # noqa: E402
from selkies_gstreamer_amd.ops.native import PinnedBuffer, require_gpu  # noqa: E402
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop  # noqa: E402

CASES = [("h264", pixelflux.OUTPUT_MODE_H264, 1920, 1080), ("hevc", pixelflux.OUTPUT_MODE_HEVC, 3840, 2160),
         ("av1", pixelflux.OUTPUT_MODE_AV1, 3840, 2160)]


def run(name, mode, W, H, before=20, after=20, fps=60.0):
    src = SyntheticDesktop(W, H, kind="motion", seed=3)
    pool = PinnedBuffer((8, H, W, 4))
    for i in range(8):
        src.frame(i, out=pool.array[i])
    s = pixelflux.default_settings(W, H, use_cpu=0, source=pixelflux.SOURCE_POOL, step_mode=1, pool_frames=8,
                                   pool_stride=W * 4, stripe_height=64, use_paint_over_quality=0,
                                   output_mode=mode, h264_fullframe=int(mode != pixelflux.OUTPUT_MODE_H264))
    s.pool = pool.array.ctypes.data
    cap = pixelflux.ScreenCapture()
    keys = []

    def on_frame(res, n, user):
        keys.append(any(res[i].size > 1 and res[i].data[1] == 1 for i in range(n)))   # header byte 1: key
    cb = pixelflux.FrameCallback(on_frame)
    cap.start_frame_capture(s, cb)

    def paced(k):   # one frame granted every 1/fps s, as a live source
        t0 = time.perf_counter()
        for i in range(k):
            while time.perf_counter() < t0 + i / fps:
                time.sleep(0.0005)
            cap.run(1)
        assert cap.wait(120_000) == 0
    try:
        paced(before)
        lat_before = cap.latencies(reset=True)
        t0 = time.perf_counter()
        res = cap.move_to(0, 20_000)
        move_ms = (time.perf_counter() - t0) * 1e3
        paced(after)
        lat_after = cap.latencies(reset=True)
        st = cap.stats()
    finally:
        cap.close()
    return {"codec": name, "resolution": f"{W}x{H}", "result": res,
            "move_stall_ms": round(st["move_stall_ms"], 3), "move_to_call_ms": round(move_ms, 2),
            "latency_before_p50_ms": round(float(np.percentile(lat_before[-before // 2:], 50)), 3),
            "first_frame_after_ms": round(float(lat_after[0]), 3),
            "latency_after_max_ms": round(float(max(lat_after)), 3),
            "latency_after_p50_ms": round(float(np.percentile(lat_after, 50)), 3),
            "key_frames_after_move": int(sum(keys[before:]))}


def main():
    require_gpu()
    for c in CASES:
        print(json.dumps(run(*c)), flush=True)


if __name__ == "__main__":
    main()
