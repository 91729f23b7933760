"""Generates csrc/codec/av1_tables.h: the normative AV1 default CDFs, quantizer
lookup tables and smooth-prediction weights the encoder needs.

Provenance. These are data tables of the AV1 specification (Default_*_Cdf,
Dc_Qlookup / Ac_Qlookup, Sm_Weights_*). The spec text is not on this image and
there is no network, but the image ships dav1d 1.5.3 + libaom 3.13.2 inside
Pillow's libavif (pillow.libs/libavif-*.so), whose read-only data holds the same
tables. This tool reads them from that file (nothing is executed):

  * large tables come from libaom's arrays (AOM_CDFn layout: N inverted values
    ending in 0, then a 0 adaptation counter, arrays padded to CDF_SIZE of the
    widest member), each located by the byte signature of its first row;
  * the small binary tables that libaom folds into code are taken from known
    values and must appear verbatim in dav1d's default-CDF struct (pairs of
    inverted value + counter) — a mismatch aborts generation;
  * every CDF is checked: strictly increasing, ending at 32768, correct counts.

The generated header is committed; the encoder's streams are then verified by
decoding them with dav1d itself (tests/test_av1_encoder.py), which is the real
check on every table used.

    python tools/av1/extract_tables.py [--lib path] > csrc/codec/av1_tables.h
"""
from __future__ import annotations

import argparse
import glob
import os
import sys

import numpy as np


def find_lib():
    import PIL
    base = os.path.dirname(os.path.dirname(PIL.__file__))
    hits = sorted(glob.glob(os.path.join(base, "pillow.libs", "libavif*.so*")))
    if not hits:
        sys.exit("libavif (with libaom/dav1d) not found")
    return hits[0]


class Image:
    def __init__(self, path):
        self.b = open(path, "rb").read()
        self.u16 = np.frombuffer(self.b[:len(self.b) // 2 * 2], dtype="<u2")

    def find(self, vals, dtype="<u2"):
        pat = np.array(vals, dtype=dtype).tobytes()
        out, i = [], self.b.find(pat)
        while i >= 0:
            out.append(i)
            i = self.b.find(pat, i + 1)
        return out

    def aom_table(self, first, count, stride, nsyms):
        """libaom array located by its first CDF (spec-form values, without 32768).
        nsyms: int or list (per group). Returns list of spec-form CDFs (N values)."""
        # `first`: the first row's leading values, or several complete rows (list of lists)
        rows = first if isinstance(first[0], list) else [first]
        n0 = nsyms[0] if isinstance(nsyms, list) else nsyms
        sig = []
        for r in rows:
            sig += [32768 - v for v in r] + ([0] * (stride - len(r)) if len(r) == n0 - 1 else [])
        hits = [h for h in self.find(sig) if h % 2 == 0]
        if not hits:
            raise SystemExit(f"signature {first} not found")
        off = hits[0] // 2
        out = []
        for g in range(count):
            n = nsyms[g] if isinstance(nsyms, list) else nsyms
            raw = self.u16[off + g * stride: off + g * stride + stride].tolist()
            vals = [32768 - x for x in raw[:n - 1]] + [32768]
            if raw[n - 1] != 0 or raw[n] != 0:
                raise SystemExit(f"table at {first}: group {g} is not an N={n} CDF: {raw}")
            check(vals, n, f"{first}[{g}]")
            out.append(vals)
        return out

    def aom_table_at(self, byte_off, count, stride, n):
        off = byte_off // 2
        out = []
        for g in range(count):
            raw = self.u16[off + g * stride: off + g * stride + stride].tolist()
            vals = [32768 - x for x in raw[:n - 1]] + [32768]
            if raw[n - 1] != 0 or raw[n] != 0:
                raise SystemExit(f"table at {byte_off}: group {g} is not an N={n} CDF: {raw}")
            check(vals, n, f"@{byte_off}[{g}]")
            out.append(vals)
        return out

    def aom_struct(self, first, layout):
        """A libaom struct of consecutive CDF_SIZE(n) members: layout = [(count, n)]."""
        sig = [32768 - v for v in first]
        hits = [h for h in self.find(sig) if h % 2 == 0]
        if not hits:
            raise SystemExit(f"signature {first} not found")
        off = hits[0] // 2
        out = []
        for count, n in layout:
            grp = []
            for _ in range(count):
                raw = self.u16[off: off + n + 1].tolist()
                vals = [32768 - x for x in raw[:n - 1]] + [32768]
                if raw[n - 1] != 0 or raw[n] != 0:
                    raise SystemExit(f"struct at {first}: not an N={n} CDF: {raw}")
                check(vals, n, f"{first}+{off}")
                grp.append(vals)
                off += n + 1
            out.append(grp)
        return out

    def confirm_binary(self, name, probs):
        """Small binary tables: must occur in dav1d's default CDF struct."""
        pat = []
        for p in probs:
            pat += [32768 - p, 0]
        if not self.find(pat):
            raise SystemExit(f"{name} {probs} not found in the dav1d tables")
        return [[p, 32768] for p in probs]


def check(vals, n, what):
    if len(vals) != n or vals[-1] != 32768:
        raise SystemExit(f"{what}: bad CDF {vals}")
    if any(b <= a for a, b in zip(vals, vals[1:])) or vals[0] <= 0:
        raise SystemExit(f"{what}: not strictly increasing {vals}")


def fmt_cdf(vals, width):
    """spec-form CDF padded to `width` u16: values, then counter 0, then 0 padding."""
    row = list(vals) + [0] * (width - len(vals))
    return "{" + ", ".join(str(v) for v in row) + "}"


def nest(rows, dims):
    """rows: flat list of strings; dims: outer dims -> nested C initializer."""
    if not dims:
        assert len(rows) == 1
        return rows[0]
    step = len(rows) // dims[0]
    return "{" + ", ".join(nest(rows[i * step:(i + 1) * step], dims[1:]) for i in range(dims[0])) + "}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    img = Image(a.lib or find_lib())
    T = {}   # name -> (flat CDF list, outer dims, width)

    def put(name, cdfs, dims, width):
        assert int(np.prod(dims)) == len(cdfs), (name, dims, len(cdfs))
        T[name] = (cdfs, dims, width)

    # ---- mode info (libaom entropymode.c arrays)
    put("kf_y_mode", img.aom_table([15588, 17027, 19338, 20218, 20682, 21110, 21825, 23244, 24189, 28165, 29093, 30466],
                                   25, 14, 13), [5, 5], 14)
    put("y_mode", img.aom_table([22801, 23489, 24293, 24756, 25601, 26123], 4, 14, 13), [4], 14)
    uv = img.aom_table([22631, 24152, 25378, 25661, 25986, 26520], 26, 15, [13] * 13 + [14] * 13)
    put("uv_mode_cfl_not_allowed", uv[:13], [13], 15)
    put("uv_mode_cfl_allowed", uv[13:], [13], 15)
    put("angle_delta", img.aom_table([2180, 5032, 7567, 22776, 26989, 30217], 8, 8, 7), [8], 8)
    part = img.aom_table([19132, 25510, 30392], 20, 11, [4] * 4 + [10] * 12 + [8] * 4)
    put("partition_w8", part[0:4], [4], 11)
    put("partition_w16", part[4:8], [4], 11)
    put("partition_w32", part[8:12], [4], 11)
    put("partition_w64", part[12:16], [4], 11)
    put("partition_w128", part[16:20], [4], 11)
    # intra_ext_tx[3 sets][4 sizes][13 modes][17]: set 1 = 7 types, set 2 = 5 types
    s1 = img.aom_table([1535, 8035, 9461, 12751, 23467, 27825], 52, 17, 7)
    # set 2 directly follows set 1 (its first rows are uniform, so locate it from set 1)
    s1_off = img.find([32768 - v for v in [1535, 8035, 9461, 12751, 23467, 27825]] + [0, 0])[0]
    s2 = img.aom_table_at(s1_off + 52 * 34, 52, 17, 5)
    put("intra_tx_set1", s1, [4, 13], 8)
    put("intra_tx_set2", s2, [4, 13], 6)
    s1i = img.aom_table([4458, 5560, 7695, 9709, 13330, 14789], 4, 17, 16)
    s1i_off = img.find([32768 - v for v in [4458, 5560, 7695, 9709, 13330, 14789]])[0]
    s3i = img.aom_table_at(s1i_off + 2 * 136, 4, 17, 2)
    put("inter_tx_set1", s1i, [4], 17)
    put("inter_tx_set3", s3i, [4], 3)
    put("single_ref", img.aom_table([[4897], [1555], [4236], [8650]], 18, 3, 2), [3, 6], 3)
    # ---- small binary tables (values confirmed against dav1d's struct)
    put("skip", img.confirm_binary("skip", [31671, 16515, 4576]), [3], 3)
    put("intra_inter", img.confirm_binary("intra_inter", [806, 16662, 20186, 26538]), [4], 3)
    put("newmv", img.confirm_binary("newmv", [24035, 16630, 15339, 8386, 12222, 4676]), [6], 3)
    put("zeromv", img.confirm_binary("zeromv", [2175, 1054]), [2], 3)
    put("refmv", img.confirm_binary("refmv", [23974, 24188, 17848, 28622, 24312, 19923]), [6], 3)
    put("drl", img.confirm_binary("drl", [13104, 24560, 18945]), [3], 3)
    dq = [28160, 32120, 32677, 32768]
    if not img.find([32768 - v for v in dq[:3]] + [0, 0]):
        raise SystemExit("delta_q cdf not found")
    put("delta_q", [dq], [1], 5)
    # ---- palette (screen content tools, key frames): has_palette_y [bsize ctx 7][neighbour
    # ctx 3] and has_palette_uv [2] are binary (confirmed in dav1d's struct), the size CDF
    # [7] and the luma colour-index CDFs [size 2..8][5 contexts] are libaom arrays (the
    # index table's rows have 2..8 symbols at a 9-entry stride)
    put("palette_y_mode", img.confirm_binary("palette_y_mode", [31676, 3419, 1261, 31912, 2859, 980, 31823, 3400, 781,
                                                                  32030, 3561, 904, 32309, 7337, 1462, 32265, 4015, 1521,
                                                                  32450, 7946, 129]), [7, 3], 3)
    put("palette_uv_mode", img.confirm_binary("palette_uv_mode", [32461, 21488]), [2], 3)
    put("palette_y_size", img.aom_table([7952, 13000, 18149, 21478, 25527, 29241], 7, 8, 7), [7], 8)
    put("palette_y_color", img.aom_table([[28710], [16384], [10553], [27036], [31603]], 35, 9,
                                         [n for n in range(2, 9) for _ in range(5)]), [7, 5], 9)
    # ---- motion vectors (libaom nmv_context: joints, then two nmv_component structs)
    mv = img.aom_struct([4096, 11264, 19328], [(1, 4), (1, 11), (2, 4), (1, 4), (1, 2), (1, 2), (1, 2), (1, 2), (10, 2),
                                               (1, 11), (2, 4), (1, 4), (1, 2), (1, 2), (1, 2), (1, 2), (10, 2)])
    put("mv_joint", mv[0], [1], 5)
    for c in range(2):
        g = mv[1 + 8 * c: 9 + 8 * c]
        put(f"mv{c}_classes", g[0], [1], 12)
        put(f"mv{c}_class0_fp", g[1], [2], 5)
        put(f"mv{c}_fp", g[2], [1], 5)
        put(f"mv{c}_sign", g[3], [1], 3)
        put(f"mv{c}_class0_hp", g[4], [1], 3)
        put(f"mv{c}_hp", g[5], [1], 3)
        put(f"mv{c}_class0", g[6], [1], 3)
        put(f"mv{c}_bits", g[7], [10], 3)
    # ---- coefficients (libaom token_cdfs.h), per quantizer context [4]
    put("txb_skip", img.aom_table([[31849], [5892], [12112], [21935]], 260, 3, 2), [4, 5, 13], 3)
    put("eob_extra", img.aom_table([[16961], [17223], [7621]], 360, 3, 2), [4, 5, 2, 9], 3)
    put("dc_sign", img.aom_table([[16000], [13056], [18816], [15232]], 24, 3, 2), [4, 2, 3], 3)
    eobs = {}
    # eob_multi{16..1024}[4][2][2]: located as one run starting with the 1024 table
    off = img.find([32768 - v for v in [393, 421, 751, 1623]])[0] // 2
    for n, name in ((11, "eob_pt_1024"), (10, "eob_pt_512"), (9, "eob_pt_256"), (8, "eob_pt_128"), (7, "eob_pt_64"),
                    (6, "eob_pt_32"), (5, "eob_pt_16")):
        cdfs = []
        for g in range(16):
            raw = img.u16[off + g * (n + 1): off + (g + 1) * (n + 1)].tolist()
            vals = [32768 - x for x in raw[:n - 1]] + [32768]
            if raw[n - 1] != 0 or raw[n] != 0:
                raise SystemExit(f"{name} group {g} bad: {raw}")
            check(vals, n, name)
            cdfs.append(vals)
        off += 16 * (n + 1)
        eobs[name] = cdfs
    for name, cdfs in eobs.items():
        n = len(cdfs[0])
        if name in ("eob_pt_512", "eob_pt_1024"):   # spec: [qctx][ptype] (libaom's 2nd ctx is unused)
            put(name, [cdfs[i] for i in range(16) if i % 2 == 0], [4, 2], n + 1)
        else:
            put(name, cdfs, [4, 2, 2], n + 1)
    put("coeff_base_eob", img.aom_table([[17837, 29055], [29600, 31446]], 160, 4, 3), [4, 5, 2, 4], 4)
    base_br = img.aom_table([[4034, 8930, 12727], [18082, 29741, 31877]], 2520, 5, 4)
    put("coeff_base", base_br[:1680], [4, 5, 2, 42], 5)
    put("coeff_br", base_br[1680:], [4, 5, 2, 21], 5)

    # ---- non-CDF tables
    dcq = img.find([4, 8, 8, 9, 10, 11, 12, 12, 13, 14], "<i2")[0] // 2
    acq = img.find([4, 8, 9, 10, 11, 12, 13, 14, 15, 16], "<i2")[0] // 2
    dc = np.frombuffer(img.b[dcq * 2: dcq * 2 + 512], dtype="<i2").tolist()
    ac = np.frombuffer(img.b[acq * 2: acq * 2 + 512], dtype="<i2").tolist()
    assert dc[-1] == 1336 and ac[-1] == 1828 and all(b >= a for a, b in zip(dc, dc[1:])) \
        and all(b >= a for a, b in zip(ac, ac[1:])), "qlookup"
    smo = img.find([0, 0, 255, 128, 255, 149, 85, 64, 255, 197, 146, 105], "u1")[0]
    sm = list(img.b[smo: smo + 128])
    assert sm[2:4] == [255, 128] and sm[64] == 255 and sm[127] > 0, "smooth weights"

    out = []
    w = out.append
    w("// GENERATED by tools/av1/extract_tables.py -- do not edit.")
    w("// AV1 normative default CDFs (spec form: cumulative x32768, last value 32768,")
    w("// then the adaptation counter, zero-padded to the row width), 8-bit quantizer")
    w("// lookups and smooth-prediction weights. See the tool for provenance/checks.")
    w("#pragma once")
    w("#include <stdint.h>")
    w('#include "sk_common.h"')
    w("")
    w("namespace sk::av1 {")
    w("")
    mode_names = [k for k in T if k not in ("txb_skip", "eob_extra", "dc_sign", "coeff_base_eob", "coeff_base",
                                            "coeff_br") and not k.startswith("eob_pt")]
    coef_names = ["txb_skip", "eob_extra", "dc_sign", "eob_pt_16", "eob_pt_32", "eob_pt_64", "eob_pt_128",
                  "eob_pt_256", "eob_pt_512", "eob_pt_1024", "coeff_base_eob", "coeff_base", "coeff_br"]
    # one CdfContext = mode part + the coefficient part of one quantizer context
    w("// The adaptive state of one tile: every CDF the encoder codes with.")
    w("struct CdfContext {")
    for k in mode_names:
        cdfs, dims, width = T[k]
        d = "".join(f"[{x}]" for x in dims)
        w(f"    uint16_t {k}{d}[{width}];")
    for k in coef_names:
        cdfs, dims, width = T[k]
        d = "".join(f"[{x}]" for x in dims[1:])
        w(f"    uint16_t {k}{d}[{width}];")
    w("};")
    w("")
    w("// Default contexts for the four coefficient quantizer contexts (qindex <= 20,")
    w("// <= 60, <= 120, else); the mode part is the same in all four.")
    w("SK_TABLE CdfContext AV1_DEFAULT_CDF[4] = {")
    for q in range(4):
        parts = []
        for k in mode_names:
            cdfs, dims, width = T[k]
            parts.append(nest([fmt_cdf(c, width) for c in cdfs], dims))
        for k in coef_names:
            cdfs, dims, width = T[k]
            per = len(cdfs) // 4
            parts.append(nest([fmt_cdf(c, width) for c in cdfs[q * per:(q + 1) * per]], dims[1:]))
        w("    {" + ",\n     ".join(parts) + "},")
    w("};")
    w("")
    w("SK_TABLE int16_t AV1_DC_QLOOKUP[256] = {" + ", ".join(map(str, dc)) + "};")
    w("SK_TABLE int16_t AV1_AC_QLOOKUP[256] = {" + ", ".join(map(str, ac)) + "};")
    w("// Sm_Weights_Tx_4x4 .. 64x64 concatenated: weights for size n start at index n.")
    w("SK_TABLE uint8_t AV1_SM_WEIGHTS[128] = {" + ", ".join(map(str, sm)) + "};")
    w("")
    w("}  // namespace sk::av1")
    print("\n".join(out))


if __name__ == "__main__":
    main()
