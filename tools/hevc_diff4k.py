"""Diagnostic: HIP vs CPU HEVC encoders on one content / size; prints the first units whose
CU decisions or levels differ (tests/test_hevc_gpu.py asserts only that they are equal)."""
import sys
import numpy as np
sys.path.insert(0, '.')
from selkies_gstreamer_amd.ops.native import HevcEncoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop

W, H = int(sys.argv[1]), int(sys.argv[2])
kind = sys.argv[3] if len(sys.argv) > 3 else "desktop"
frames = int(sys.argv[4]) if len(sys.argv) > 4 else 2
gpu = HevcEncoder(W, H, backend="hip", device=0)
cpu = HevcEncoder(W, H, backend="cpu")
src = SyntheticDesktop(W, H, kind=kind)
W16 = (W + 15) // 16
for t in range(frames):
    f = src.frame(t)
    pg, pc = gpu.encode(f, t), cpu.encode(f, t)
    cg = np.frombuffer(gpu.debug_buffer("cus", np.uint8), np.uint8).reshape(-1, 40)
    cc = np.frombuffer(cpu.debug_buffer("cus", np.uint8), np.uint8).reshape(-1, 40)
    lg = np.frombuffer(gpu.debug_buffer("coefs", np.uint8), np.int16).reshape(-1, 384)
    lc = np.frombuffer(cpu.debug_buffer("coefs", np.uint8), np.int16).reshape(-1, 384)
    dc = np.nonzero((cg != cc).any(axis=1))[0]
    dl = np.nonzero((lg != lc).any(axis=1))[0]
    print(f"frame {t}: packets equal {[p.data for p in pg] == [p.data for p in pc]} sizes {len(pg[0].data)} {len(pc[0].data)}; "
          f"cu diffs {len(dc)}, level diffs {len(dl)}", flush=True)
    for i in list(dc[:4]):
        print("  unit", i, "xy", i % W16, i // W16, "\n   gpu", cg[i].tolist(), "\n   cpu", cc[i].tolist())
    for i in list(dl[:3]):
        d = np.nonzero(lg[i] != lc[i])[0]
        print("  levels unit", i, "xy", i % W16, i // W16, "first idx", d[:8].tolist(), lg[i][d[:8]].tolist(), lc[i][d[:8]].tolist())
    if [p.data for p in pg] != [p.data for p in pc]:
        from selkies_gstreamer_amd.models.hevc.decoder import split_annexb
        ng, nc = split_annexb(pg[0].data[10:]), split_annexb(pc[0].data[10:])
        print("  nals", len(ng), len(nc))
        for k, (a, b) in enumerate(zip(ng, nc)):
            if a != b:
                d = next(i for i in range(min(len(a), len(b))) if a[i] != b[i]) if len(a) == len(b) else -1
                print(f"  nal {k}: type {(a[0] >> 1) & 63} len {len(a)} {len(b)} first diff byte {d}",
                      a[max(0, d - 4):d + 8].hex(), b[max(0, d - 4):d + 8].hex())
        sg = np.frombuffer(gpu.debug_buffer("sao", np.uint8), np.uint8).reshape(-1, 28)
        sc = np.frombuffer(cpu.debug_buffer("sao", np.uint8), np.uint8).reshape(-1, 28)
        ds = np.nonzero((sg != sc).any(axis=1))[0]
        print("  sao diffs", len(ds), ds[:5].tolist())
        bg = np.frombuffer(gpu.debug_buffer("bin_n", np.uint8), np.int32)
        bc = np.frombuffer(cpu.debug_buffer("bin_n", np.uint8), np.int32) if True else None
        db = np.nonzero(bg != bc)[0]
        print("  bin_n diffs", len(db), db[:8].tolist(), bg[db[:8]].tolist(), bc[db[:8]].tolist())
