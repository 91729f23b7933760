"""Key-frame cost of one session of any codec: a key frame requested every `period` frames
after warm-up; prints host-side encode times of key vs inter frames and their sizes. Run
under `rocprofv3 --kernel-trace --stats` (tools/gpu.sh profpy) for the kernel durations.

    python tools/key_latency.py --codec hevc --width 3840 --height 2160 --rc cbr --kbps 20000
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selkies_gstreamer_amd.ops.native import H264Encoder  # noqa: E402
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--codec", default="hevc")
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--frames", type=int, default=40)
ap.add_argument("--period", type=int, default=4)
ap.add_argument("--rc", default="crf")
ap.add_argument("--kbps", type=int, default=0)
ap.add_argument("--fps", type=float, default=60.0)
ap.add_argument("--content", default="motion")
ap.add_argument("--tiles", default="-1,-1", help="AV1 tile_cols_log2,tile_rows_log2 (-1: automatic)")
a = ap.parse_args()
src = SyntheticDesktop(a.width, a.height, a.content, seed=7)
pool = [src.frame(i) for i in range(8)]
enc = H264Encoder(a.width, a.height, codec=a.codec, fullframe=True, backend="hip", fps=a.fps, rate_control=a.rc,
                  bitrate_kbps=a.kbps, use_paint_over=False,
                  tile_cols_log2=int(a.tiles.split(",")[0]), tile_rows_log2=int(a.tiles.split(",")[1]))
key, inter = [], []
for t in range(a.frames):
    want_key = t >= 10 and t % a.period == 0
    if want_key:
        enc.request_keyframe()
    t0 = time.perf_counter()
    pk = enc.encode(pool[t % len(pool)], t)
    dt = (time.perf_counter() - t0) * 1e3
    nb = sum(len(p.data) for p in pk)
    is_key = any(p.key for p in pk)
    if t >= 10:
        (key if is_key else inter).append((dt, nb / 1024))
    print(f"frame {t:3d} {'K' if is_key else 'P'} {dt:7.3f} ms {nb / 1024:8.1f} KiB", flush=True)
enc.close()
for name, v in (("key", key), ("inter", inter)):
    if v:
        d = np.array(v)
        print(f"{name:5s} frames: n={len(v)} median {np.median(d[:, 0]):.3f} ms max {d[:, 0].max():.3f} ms, "
              f"median {np.median(d[:, 1]):.1f} KiB")
