#!/usr/bin/env python3
"""Per-kernel summary (markdown) of a rocprofv3 --kernel-trace database.

    python tools/prof_summary.py gpurun_out/<dir>/run_results.db "title" > profiles/<name>.md
"""
import sqlite3
import sys

import numpy as np


def main(path: str, title: str = "") -> None:
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(rocpd_kernel_dispatch)")]
    sym = {r[0]: r[1] for r in db.execute("select id, display_name from rocpd_info_kernel_symbol")}
    rows = db.execute("select kernel_id, start, end, grid_size_x, grid_size_y, workgroup_size_x, "
                      "workgroup_size_y from rocpd_kernel_dispatch").fetchall()
    ks = {}
    for kid, st, en, gx, gy, wx, wy in rows:
        name = sym.get(kid, str(kid)).split("(")[0].replace("sk::h264::gpu::", "").replace("sk::jpeg::gpu::", "")
        name = name.replace("void ", "")
        d = ks.setdefault(name, {"t": [], "grid": (gx * gy) // max(1, wx * wy), "wg": wx * wy})
        d["t"].append((en - st) / 1e3)
    tot = sum(sum(d["t"]) for d in ks.values())
    print(f"# {title}\n\nsource: `{path}`\n")
    print("| kernel | calls | total ms | share | median us | p90 us | max us | blocks | wg |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, d in sorted(ks.items(), key=lambda kv: -sum(kv[1]["t"])):
        t = np.array(d["t"])
        print(f"| {name} | {len(t)} | {t.sum() / 1e3:.2f} | {100 * t.sum() / tot:.1f}% | {np.median(t):.1f} | "
              f"{np.percentile(t, 90):.1f} | {t.max():.1f} | {d['grid']} | {d['wg']} |")
    _ = cols


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
