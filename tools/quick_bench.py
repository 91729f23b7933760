"""Quick single-session timing of the HIP H.264 pipeline (dev tool)."""
import sys, time
import numpy as np
sys.path.insert(0, ".")
from selkies_gstreamer_amd.ops.native import H264Encoder
from tests.h264_util import synthetic_frames

W, H = 1920, 1080
kind = sys.argv[1] if len(sys.argv) > 1 else "desktop"
frames = list(synthetic_frames(W, H, 16, seed=1, kind=kind))
for ff in (False, True):
    enc = H264Encoder(W, H, stripe_height=64, fullframe=ff, qp=25, backend="hip")
    for t in range(5):
        enc.encode(frames[t % 16], t)
    n = 60
    ts = []
    nbytes = 0
    t0 = time.perf_counter()
    for t in range(n):
        a = time.perf_counter()
        pk = enc.encode(frames[t % 16], t)
        ts.append(time.perf_counter() - a)
        nbytes += sum(len(p.data) for p in pk)
    el = time.perf_counter() - t0
    print(f"{kind} fullframe={ff}: {n/el:.1f} fps, p50 {1e3*np.median(ts):.2f} ms, "
          f"p99 {1e3*np.percentile(ts,99):.2f} ms, {nbytes/n/1024:.1f} KiB/frame, stages(us)={enc.stage_times()}")
