"""Steady-state keyframe cost: one 1080p H.264 session, a keyframe requested every
`period` frames after warm-up. Prints the host-side encode time of IDR vs P frames;
run under `rocprofv3 --kernel-trace --stats` for the k_code_intra durations."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selkies_gstreamer_amd.ops.native import H264Encoder  # noqa: E402
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop  # noqa: E402

W, H = 1920, 1080
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 60
period = int(sys.argv[2]) if len(sys.argv) > 2 else 4
kind = sys.argv[3] if len(sys.argv) > 3 else "motion"
intra4x4 = len(sys.argv) > 4 and sys.argv[4] == "i4"
src = SyntheticDesktop(W, H, kind)
pool = [src.frame(i) for i in range(8)]
enc = H264Encoder(W, H, stripe_height=64, backend="hip", use_paint_over=False, intra4x4=intra4x4)
idr, p, idr_bytes = [], [], []
for t in range(frames):
    key = t >= 10 and t % period == 0
    if key:
        enc.request_keyframe()
    t0 = time.perf_counter()
    pk = enc.encode(pool[t % len(pool)], t)
    dt = (time.perf_counter() - t0) * 1e3
    if t >= 10:
        (idr if key else p).append(dt)
        if key:
            idr_bytes.append(sum(len(x.data) for x in pk))
print(f"IDR frames: n={len(idr)} median {np.median(idr):.3f} ms max {max(idr):.3f} ms, "
      f"median {np.median(idr_bytes) / 1024:.1f} KiB (intra4x4={intra4x4})")
print(f"P frames:   n={len(p)} median {np.median(p):.3f} ms max {max(p):.3f} ms")
