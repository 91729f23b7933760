"""Where the HIP HEVC back end first departs from the CPU reference: CU records (24-byte
CuInfo) and levels of one key frame, printed field by field. Debug aid for kernel changes."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from selkies_gstreamer_amd.ops.native import HevcEncoder  # noqa: E402
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (128, 64)
src = SyntheticDesktop(W, H, kind="motion")
encs = {b: HevcEncoder(W, H, backend=b, **({"device": 0} if b == "hip" else {})) for b in ("hip", "cpu")}
f = src.frame(0)
for e in encs.values():
    e.encode(f, 0)
cu = {b: np.frombuffer(e.debug_buffer("cus", np.uint8), np.uint8).reshape(-1, 24) for b, e in encs.items()}
lv = {b: np.frombuffer(e.debug_buffer("coefs", np.uint8), np.int16).reshape(-1, 384) for b, e in encs.items()}
names = ["mode", "merge", "mvp", "imode", "cbf", "qp", "tu", "tuc"]
bad = np.nonzero((cu["hip"] != cu["cpu"]).any(1))[0]
print("differing CUs:", len(bad), "of", len(cu["cpu"]), bad[:20])
for i in bad[:6]:
    g, c = cu["hip"][i], cu["cpu"][i]
    d = {n: (int(g[k]), int(c[k])) for k, n in enumerate(names) if g[k] != c[k]}
    for off, n in ((16, "ycbf"), (18, "tsy")):
        a, b = int(g[off]) | int(g[off + 1]) << 8, int(c[off]) | int(c[off + 1]) << 8
        if a != b:
            d[n] = (hex(a), hex(b))
    if g[20] != c[20]:
        d["tsc"] = (hex(g[20]), hex(c[20]))
    lz = np.nonzero(lv["hip"][i] != lv["cpu"][i])[0]
    print("CU", i, "hip/cpu:", d, "levels differ at", lz[:12], lv["hip"][i][lz[:6]], lv["cpu"][i][lz[:6]])
