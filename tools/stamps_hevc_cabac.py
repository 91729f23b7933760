"""Diagnostic: cycles and bin entries per CTB row of k_hevc_cabac (SK_STAMPS=1)."""
import os, sys
import numpy as np
os.environ["SK_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from selkies_gstreamer_amd.ops.native import HevcEncoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
W, H = int(sys.argv[1]) if len(sys.argv) > 1 else 3840, int(sys.argv[2]) if len(sys.argv) > 2 else 2160
src = SyntheticDesktop(W, H, "motion")
enc = HevcEncoder(W, H, backend="hip")
for t in range(3):
    enc.encode(src.frame(t), t)
st = np.frombuffer(enc.debug_buffer("hevc_stamps", np.uint8), np.uint64).reshape(-1, 4).astype(np.int64)
cwait = (st[:, 1] >> 24) & 0xFFFFF   # coder wave sleeps (ring empty)
mwait = st[:, 1] >> 44                # modeler wave sleeps (ring full)
st[:, 1] &= 0xFFFFFF
bn = np.frombuffer(enc.debug_buffer("bin_n", np.uint8), np.int32)
print("rows", len(st), "median cycles/row", np.median(st[:, 0]), "median entries/row", np.median(st[:, 1]))
rt = (st[:, 3] - st[:, 2]) / 100.0   # s_memrealtime: 100 MHz -> us
print("row duration us (realtime): median", np.median(rt), "max", rt.max(),
      "-> core MHz implied", np.median(st[:, 0] / np.maximum(rt, 1e-3)))
s0 = st[:, 2] - st[:, 2].min()
print("row start offsets us: median", np.median(s0) / 100, "max", s0.max() / 100,
      "kernel span us", (st[:, 3].max() - st[:, 2].min()) / 100)
order = np.argsort(st[:, 2])
print("first 12 rows to start:", order[:12].tolist(), "start us", (s0[order[:12]] / 100).round(1).tolist())
print("cycles per entry (median over rows):", np.median(st[:, 0] / np.maximum(st[:, 1], 1)))
print("total entries", bn.sum(), "max per CU", bn.max())
hv = np.argsort(st[:, 1])[-5:]
print("heaviest rows", hv.tolist(), "entries", st[hv, 1].tolist(), "coder waits", cwait[hv].tolist(),
      "modeler waits", mwait[hv].tolist())
print("median waits: coder", np.median(cwait), "modeler", np.median(mwait))
