"""Busy-time summary of a rocprofv3 trace with kernels and memory copies (--kernel-trace
--memory-copy-trace): over the window [t0, t1] of the last `--frac` of the dispatches, the
union of kernel intervals, of copy intervals (by direction), their overlap and the idle time,
per frame when `--frames` is given.

    python tools/timeline_summary.py gpurun_out/r6m/prof/run_results.db --frames 1600 --frac 0.8
"""
import argparse
import sqlite3


def union(iv):
    iv = sorted(iv)
    out, cs, ce = [], None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                out.append((cs, ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        out.append((cs, ce))
    return out


def total(iv):
    return sum(e - s for s, e in iv)


def inter(a, b):
    i = j = 0
    t = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            t += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--frac", type=float, default=0.8)
    ap.add_argument("--frames", type=int, default=0, help="frames encoded inside the window")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    ks = db.execute("select start, end, name from kernels order by start").fetchall()
    cs = db.execute("select start, end, size, src_agent_type, dst_agent_type from memory_copies order by start").fetchall()
    t0 = ks[int(len(ks) * (1 - a.frac))][0]
    t1 = ks[-1][1]
    clip = lambda iv: [(max(s, t0), min(e, t1)) for s, e in iv if e > t0 and s < t1]
    K = union(clip([(s, e) for s, e, n in ks if "touch_pages" not in n]))
    h2d = union(clip([(s, e) for s, e, z, sa, da in cs if sa == "CPU" and da == "GPU"]))
    d2h = union(clip([(s, e) for s, e, z, sa, da in cs if sa == "GPU" and da == "CPU"]))
    nbytes = sum(z for s, e, z, sa, da in cs if sa == "CPU" and da == "GPU" and e > t0 and s < t1)
    W = t1 - t0
    C = union(h2d + d2h)
    anyb = union(K + C)
    f = a.frames * a.frac if a.frames else 0
    rows = [("window", W), ("kernels busy (union)", total(K)), ("H2D copies busy", total(h2d)),
            ("D2H copies busy", total(d2h)), ("kernels and copies overlapped", inter(K, C)),
            ("GPU idle (neither)", W - total(anyb))]
    print("| quantity | ms | % of window |" + (" us / frame |" if f else ""))
    print("|---|---|---|" + ("---|" if f else ""))
    for name, v in rows:
        print(f"| {name} | {v / 1e6:.2f} | {100 * v / W:.1f} |" + (f" {v / 1e3 / f:.1f} |" if f else ""))
    print(f"\nH2D bytes in the window: {nbytes / 1e9:.2f} GB, {nbytes / (total(h2d) or 1):.2f} GB/s while copying, "
          f"{nbytes / W:.2f} GB/s over the window")


if __name__ == "__main__":
    main()
