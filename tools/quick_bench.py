"""Single-session timing of the HIP H.264 pipeline (dev tool).
usage: python tools/quick_bench.py [motion|desktop|noise] [--idr]"""
import sys, time
import numpy as np
sys.path.insert(0, ".")
from selkies_gstreamer_amd.ops.native import H264Encoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop

W, H = 1920, 1080
kind = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "motion"
idr = "--idr" in sys.argv
src = SyntheticDesktop(W, H, kind=kind)
frames = [src.frame(t) for t in range(40)]
for ff in (False, True):
    enc = H264Encoder(W, H, stripe_height=64, fullframe=ff, qp=25, backend="hip", use_paint_over=False)
    for t in range(3):
        enc.encode(frames[t], t)
    ts, st = [], []
    nbytes = 0
    for t in range(3, 40):
        if idr:
            enc.request_keyframe()
        a = time.perf_counter()
        pk = enc.encode(frames[t], t)
        ts.append(time.perf_counter() - a)
        st.append(enc.stage_times())
        nbytes += sum(len(p.data) for p in pk)
    st = np.array(st)
    print(f"{kind} idr={idr} fullframe={ff}: p50 {1e3*np.median(ts):.2f} ms, p90 {1e3*np.percentile(ts,90):.2f} ms, "
          f"{nbytes/len(ts)/1024:.1f} KiB/frame, stage p50 us = {np.median(st, axis=0).round(1).tolist()}")
