"""Token statistics of the HIP AV1 back end (per-tile stream lengths, token kinds,
literal bits, symbol alphabet sizes): the work the per-tile arithmetic coder does.

    python tools/av1_tokstats.py --width 3840 --height 2160 [--mode cbr --kbps 40000]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frames", type=int, default=6)
    ap.add_argument("--mode", default="cqp")
    ap.add_argument("--kbps", type=int, default=0)
    ap.add_argument("--fps", type=float, default=120.0)
    ap.add_argument("--content", default="motion")
    ap.add_argument("--qp", type=int, default=25)
    ap.add_argument("--tiles", default="-1,-1", help="tile_cols_log2,tile_rows_log2 (-1: automatic)")
    a = ap.parse_args()
    from selkies_gstreamer_amd.ops.native import H264Encoder
    from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
    src = SyntheticDesktop(a.width, a.height, kind=a.content)
    enc = H264Encoder(a.width, a.height, codec="av1", fullframe=True, backend="hip", fps=a.fps,
                      rate_control=a.mode, bitrate_kbps=a.kbps, qp=a.qp,
                      tile_cols_log2=int(a.tiles.split(",")[0]), tile_rows_log2=int(a.tiles.split(",")[1]))
    for t in range(a.frames):
        pk = enc.encode(src.frame(t), t)
    nbytes = sum(len(p.data) for p in pk)
    ntok = enc.debug_buffer("tile_ntok", np.int32)
    tokc = enc.debug_buffer("tokc", np.uint32)
    cap = tokc.size // ntok.size
    kinds = np.zeros(4, np.int64)
    lit_bits = 0
    nsym = np.zeros(17, np.int64)
    for t in range(ntok.size):
        tk = tokc[t * cap: t * cap + ntok[t]]
        k = tk >> 30
        kinds += np.bincount(k, minlength=4)
        lit = tk[k == 1]
        lit_bits += int((((lit >> 25) & 31) + 1).sum())
        sy = tk[k == 0]
        nsym += np.bincount(((sy >> 26) & 15) + 1, minlength=17)
    # the busiest tile: symbols per CDF slot and per k_av1_cdf partition (same hash)
    tmax = int(ntok.argmax())
    tk = tokc[tmax * cap: tmax * cap + ntok[tmax]]
    sy = tk[(tk >> 30) != 1]
    offs, cnt = np.unique(sy & 0x3fffff, return_counts=True)
    order = np.argsort(-cnt)
    part = ((offs.astype(np.uint64) * 0x9E3779B1) & 0xFFFFFFFF) >> 28
    loads = np.bincount(part.astype(np.int64), weights=cnt, minlength=16)
    # the critical path of k_av1_cdf: the largest per-wave symbol load over all tiles
    # and its serial steps when a run of identical tokens in one wave's stream costs one
    # step (the k_av1_cdf run path; runs are cut at 64-token sub-batches)
    crit, crit_top, crit_runs = 0, 0, 0
    for t in range(ntok.size):
        tt = tokc[t * cap: t * cap + ntok[t]]
        idx = np.nonzero((tt >> 30) != 1)[0]
        full = tt[idx]
        st = full & 0x3fffff
        if st.size == 0:
            continue
        o, c = np.unique(st, return_counts=True)
        pa = ((o.astype(np.uint64) * 0x9E3779B1) & 0xFFFFFFFF) >> 28
        crit = max(crit, int(np.bincount(pa.astype(np.int64), weights=c, minlength=16).max()))
        crit_top = max(crit_top, int(c.max()))
        owner = (((st.astype(np.uint64) * 0x9E3779B1) & 0xFFFFFFFF) >> 28).astype(np.int64)
        for p_ in range(16):
            sel = owner == p_
            w, pos = full[sel], idx[sel]
            if w.size:
                head = np.ones(w.size, bool)
                head[1:] = (w[1:] != w[:-1]) | (pos[1:] // 64 != pos[:-1] // 64)
                crit_runs = max(crit_runs, int(head.sum()))
    out = {"cdf_critical_symbols": crit, "cdf_critical_run_heads": crit_runs, "cdf_hottest_context_symbols": crit_top,
           "max_tile_contexts": int(offs.size),
           "max_tile_top_contexts": [[int(offs[i]), int(cnt[i])] for i in order[:12]],
           "max_tile_partition_loads": [int(x) for x in loads],
           "width": a.width, "height": a.height, "mode": a.mode, "kbps": a.kbps, "frame_bytes": nbytes,
           "tiles": int(ntok.size), "tokens_total": int(ntok.sum()), "tokens_max_tile": int(ntok.max()),
           "tokens_mean_tile": float(ntok.mean()), "symbols": int(kinds[0]), "literal_tokens": int(kinds[1]),
           "literal_bits": lit_bits, "gathers": int(kinds[2] + kinds[3]),
           "symbols_by_N": {int(n): int(c) for n, c in enumerate(nsym) if c}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
