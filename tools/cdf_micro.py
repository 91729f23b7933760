"""k_av1_cdf in isolation: replays the busiest tile's token stream of a real AV1 frame
(or a filtered copy of it) through the test entry sk_av1_ec_tokens_hip, `--reps` times,
so `rocprofv3 --kernel-trace --stats` (tools/gpu.sh profpy) times the kernel alone.

    python tools/cdf_micro.py --variant tile|hot|nohot [--frames 1] [--reps 5] [--libs a.so,b.so]

With --libs the test entry of each library (e.g. builds of two versions of
av1_kernels.hip, tools/ab/) runs `--reps` times in turn, in the order given.

frame: every tile of the frame (the encoder's launch: tiles x 16 partitions)
tile:  the busiest tile of the frame as coded (16 partitions, one tile)
hot:   only the tokens of that tile's hottest context (one wave does all the work)
nohot: the tile without its hottest context
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="tile")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frames", type=int, default=1, help="1: the key frame; more: the last (inter) frame")
    ap.add_argument("--qp", type=int, default=25)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kbps", type=int, default=0, help="CBR at this rate (120 fps) instead of constant QP")
    ap.add_argument("--libs", default="", help="comma-separated libraries whose sk_av1_ec_tokens_hip to time")
    a = ap.parse_args()
    from selkies_gstreamer_amd.ops.native import H264Encoder, lib
    from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
    src = SyntheticDesktop(a.width, a.height, kind="motion")
    enc = H264Encoder(a.width, a.height, codec="av1", fullframe=True, backend="hip", qp=a.qp, fps=120.0,
                      rate_control="cbr" if a.kbps else "cqp", bitrate_kbps=a.kbps)
    for t in range(a.frames):
        enc.encode(src.frame(t), t)
    ntok = enc.debug_buffer("tile_ntok", np.int32)
    tokc = enc.debug_buffer("tokc", np.uint32)
    qidx = int(enc.debug_buffer("frame", np.int32)[1])
    enc.close()
    cap = tokc.size // ntok.size
    t = int(ntok.argmax())
    tk = tokc[t * cap: t * cap + ntok[t]].copy()
    sym = (tk >> 30) != 1
    offs, cnt = np.unique(tk[sym] & 0x3fffff, return_counts=True)
    hot = offs[cnt.argmax()]
    is_hot = sym & ((tk & 0x3fffff) == hot) & ((tk >> 30) == 0)
    if a.variant == "hot":
        tk = tk[is_hot]
    elif a.variant == "nohot":
        tk = tk[~is_hot]
    tk = np.ascontiguousarray(tk, np.uint32)
    offs_a, ns = np.zeros(1, np.int32), np.array([tk.size], np.int32)
    if a.variant == "frame":   # all tiles, each at its slot of the encoder's buffer
        tk = np.ascontiguousarray(tokc, np.uint32)
        offs_a = (np.arange(ntok.size) * cap).astype(np.int32)
        ns = ntok.astype(np.int32)
    libs = [ctypes.CDLL(x, mode=os.RTLD_LAZY | os.RTLD_LOCAL) for x in a.libs.split(",")] if a.libs else [lib()]
    for L in libs:
        run(L, tk, offs_a, ns, qidx, a.reps)
    print(f"variant {a.variant}: tokens {tk.size} (hot context {int(hot)}: {int(is_hot.sum())} of the tile's "
          f"{int(ntok[t])}), qidx {qidx}, libraries {a.libs or 'in-tree'}", flush=True)


def run(L, tk, offs_a, ns, qidx, reps):
    P = ctypes.POINTER
    L.sk_av1_ec_tokens_hip.argtypes = [P(ctypes.c_uint32), P(ctypes.c_int32), P(ctypes.c_int32), ctypes.c_int,
                                       ctypes.c_int, P(ctypes.c_uint8), ctypes.c_int, P(ctypes.c_int32),
                                       P(ctypes.c_uint32)]
    L.sk_av1_ec_tokens_hip.restype = ctypes.c_int
    out = np.zeros(8 * tk.size + 4096, np.uint8)
    sizes = np.zeros(ns.size, np.int32)
    for _ in range(reps):
        rc = L.sk_av1_ec_tokens_hip(tk.ctypes.data_as(P(ctypes.c_uint32)), offs_a.ctypes.data_as(P(ctypes.c_int32)),
                                    ns.ctypes.data_as(P(ctypes.c_int32)), ns.size, qidx,
                                    out.ctypes.data_as(P(ctypes.c_uint8)), out.size,
                                    sizes.ctypes.data_as(P(ctypes.c_int32)), None)
        assert rc == 0


if __name__ == "__main__":
    main()
