"""Quarter-pel on/off: P-frame bits and mean luma PSNR (independent decoder) on the synthetic
moving desktop, static desktop and a sub-pixel translating texture; CPU reference encoder.
usage: python tools/rd_subpel.py"""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from selkies_gstreamer_amd.ops.native import H264Encoder, ME_DTYPE
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
from tests.h264_util import StripeDecoder, bgrx_to_y709, psnr
from tests.test_h264_subpel import subpixel_scene
W, H = 640, 368
for kind in ("motion", "desktop", "subpixel"):
    frames = subpixel_scene(W, H, 16) if kind == "subpixel" else [SyntheticDesktop(W, H, kind=kind, seed=7).frame(t) for t in range(16)]
    res = {}
    for sp in (False, True):
        enc = H264Encoder(W, H, qp=25, paint_qp=25, use_paint_over=False, subpel=sp, backend="cpu")
        dec = StripeDecoder(W, H)
        bits, ps, refined = 0, [], 0
        for t, f in enumerate(frames):
            pk = enc.encode(f, t)
            if t > 0: bits += 8 * sum(len(p.data) - 10 for p in pk)
            for p in pk: dec.feed(p.data)
            ps.append(psnr(dec.Y, bgrx_to_y709(f)[:H, :W]))
            me = enc.debug_buffer("me", ME_DTYPE)
            refined += int(np.count_nonzero((me["fx"] != 0) | (me["fy"] != 0)))
        res[sp] = (bits, np.mean(ps), refined)
    print(kind, "off", res[False][:2], "on", res[True], "bits ratio", round(res[True][0] / res[False][0], 4))
