"""AV1 multi-symbol entropy coder (csrc/codec/av1_ec.h) against the independent
spec-model decoder (models/av1/entropy.py): random alphabets of 2..16 symbols,
skewed and flat CDFs, with and without adaptation, booleans and literals.
Parity with libaom/dav1d is unpinned (neither is on this image)."""
import ctypes

import numpy as np
import pytest

from selkies_gstreamer_amd.models.av1.entropy import SymbolDecoder, update_cdf


def _lib():
    from selkies_gstreamer_amd.ops import native
    L = native.lib()
    P = ctypes.POINTER
    L.sk_av1_ec_encode.argtypes = [P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_int32), ctypes.c_int,
                                   P(ctypes.c_uint16), P(ctypes.c_int32), ctypes.c_int, P(ctypes.c_uint8),
                                   ctypes.c_int]
    L.sk_av1_ec_encode.restype = ctypes.c_int
    return L


def _random_cdf(rng, n, skew):
    p = rng.dirichlet(np.full(n, skew))
    c = np.cumsum(p) * 32768
    cdf = [int(min(32767, max(1, round(x)))) for x in c[:-1]]
    for i in range(1, len(cdf)):                       # strictly increasing
        cdf[i] = max(cdf[i], cdf[i - 1] + 1)
    return cdf + [32768, 0]


def _encode(kind, ctx, sym, cdfs, nsym, adapt):
    L = _lib()
    n = len(sym)
    flat = np.zeros(len(cdfs) * 17, np.uint16)
    for c, cdf in enumerate(cdfs):
        flat[c * 17:c * 17 + len(cdf)] = cdf
    a = lambda x: (ctypes.c_int32 * len(x))(*x)   # noqa: E731
    out = (ctypes.c_uint8 * (4 * n + 64))()
    m = L.sk_av1_ec_encode(a(kind), a(ctx), a(sym), n, flat.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)),
                           a(nsym), int(adapt), out, len(out))
    assert m >= 0
    return bytes(out[:m])


@pytest.mark.parametrize("adapt", [False, True])
@pytest.mark.parametrize("seed", range(6))
def test_roundtrip_random_symbols(seed, adapt):
    rng = np.random.default_rng(seed)
    nctx = 8
    nsym = [int(rng.integers(2, 17)) for _ in range(nctx)]
    cdfs = [_random_cdf(rng, n, 0.3 if c % 2 else 3.0) for c, n in enumerate(nsym)]
    kind, ctx, sym = [], [], []
    for _ in range(3000):
        k = int(rng.choice([0, 0, 0, 1, 2]))
        if k == 0:
            c = int(rng.integers(nctx))
            # draw from the (initial) distribution so skewed contexts see skewed data
            p = np.diff([0] + cdfs[c][:nsym[c]]) / 32768
            s = int(rng.choice(nsym[c], p=p / p.sum()))
            kind.append(0), ctx.append(c), sym.append(s)
        elif k == 1:
            kind.append(1), ctx.append(0), sym.append(int(rng.integers(2)))
        else:
            bits = int(rng.integers(1, 17))
            kind.append(2), ctx.append(bits), sym.append(int(rng.integers(1 << bits)))
    data = _encode(kind, ctx, sym, [list(c) for c in cdfs], nsym, adapt)
    dec = SymbolDecoder(data)
    dcdfs = [list(c) for c in cdfs]
    for k, c, s in zip(kind, ctx, sym):
        if k == 0:
            assert dec.read_symbol(dcdfs[c], nsym[c], adapt) == s
        elif k == 1:
            assert dec.read_bool() == s
        else:
            assert dec.read_literal(c) == s
    assert dec.exit_ok()


def test_compression_tracks_entropy():
    """A skewed binary source costs close to its entropy once the CDF adapts."""
    rng = np.random.default_rng(7)
    sym = [int(x) for x in (rng.random(20000) < 0.05)]
    data = _encode([0] * len(sym), [0] * len(sym), sym, [[16384, 32768, 0]], [2], True)
    h = -(0.05 * np.log2(0.05) + 0.95 * np.log2(0.95))
    assert len(data) * 8 < 1.08 * h * len(sym)
    dec = SymbolDecoder(data)
    cdf = [16384, 32768, 0]
    assert [dec.read_symbol(cdf, 2) for _ in sym] == sym


def test_update_cdf_rule():
    cdf = [8192, 16384, 24576, 32768, 0]
    update_cdf(cdf, 4, 0)      # rate 3 + 0 + 0 + 2 = 5: every boundary moves 1/32 towards 32768
    assert cdf == [8192 + (32768 - 8192) // 32, 16384 + 16384 // 32, 24576 + 8192 // 32, 32768, 1]


def _fields(L):
    P = ctypes.POINTER
    L.sk_av1_cdf_field.argtypes = [ctypes.c_int] + [P(ctypes.c_int32)] * 4
    L.sk_av1_cdf_field.restype = ctypes.c_int
    out, i = [], 0
    while True:
        off, n, cnt, st = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        nf = L.sk_av1_cdf_field(i, off, n, cnt, st)
        if i >= nf:
            return out
        out.append((off.value, n.value, cnt.value, st.value))
        i += 1


def _token_streams(L, seed, tiles):
    """Random token streams in the av1_core.h format: adaptive symbols over a few
    reused CDFs of each default-context field (counters saturate), L(n) literals of
    1..25 bits, and gathered partition booleans; one long literal-heavy tile spans
    several carry-resolution windows of k_av1_pack."""
    rng = np.random.default_rng(seed)
    fields = _fields(L)
    part = [f for f in fields if f[1] == 10][0]          # partition_w16
    streams = []
    for t in range(tiles):
        if t == 1:   # one context, symbol 0 almost always: long runs without a resetting token
            off, ns, cnt, st = [f for f in fields if f[1] == 2][0]
            streams.append([((ns - 1) << 26) | ((1 if rng.random() < 3e-4 else 0) << 22) | off for _ in range(20000)])
            continue
        n = 12000 if t == 0 else int(rng.integers(0, 3000))
        picks = [fields[int(rng.integers(len(fields)))] for _ in range(6)]
        ctxs = [(off + int(rng.integers(cnt)) * st, ns) for off, ns, cnt, st in picks]
        toks = []
        for _ in range(n):
            k = int(rng.choice([0, 0, 0, 0, 1, 2])) if t else int(rng.choice([0, 1, 1]))
            if k == 0:
                off, ns = ctxs[int(rng.integers(len(ctxs)))]
                v = int(min(ns - 1, rng.geometric(0.5) - 1))
                toks.append(((ns - 1) << 26) | (v << 22) | off)
            elif k == 1:
                nb = int(rng.integers(1, 26))
                toks.append((1 << 30) | ((nb - 1) << 25) | int(rng.integers(1 << nb)))
            else:
                off = part[0] + int(rng.integers(part[2])) * part[3]
                toks.append((2 << 30) | (int(rng.integers(2)) << 29) | (int(rng.integers(2)) << 28) | off)
        streams.append(toks)
    return streams


def test_token_replay_cpu():
    """sk_av1_ec_tokens_cpu (the GPU coder's reference) is deterministic and sized sanely."""
    L = _lib()
    L.sk_av1_ec_tokens_cpu.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint8), ctypes.c_int]
    L.sk_av1_ec_tokens_cpu.restype = ctypes.c_int
    toks = _token_streams(L, 3, 2)[1]
    arr = (ctypes.c_uint32 * max(1, len(toks)))(*toks)
    outs = []
    for _ in range(2):
        out = (ctypes.c_uint8 * (8 * len(toks) + 64))()
        n = L.sk_av1_ec_tokens_cpu(arr, len(toks), 100, out, len(out))
        assert n > 0
        outs.append(bytes(out[:n]))
    assert outs[0] == outs[1]


@pytest.mark.gpu
def test_gpu_tiles_match_host_encoder():
    """k_av1_cdf + the block-parallel coder k_av1_ec_* (csrc/kernels/av1_kernels.hip) on
    synthetic token streams (a literal-heavy tile, a tile of long non-resetting runs, empty tiles):
    every tile byte-identical to the host replay through SymbolCoder (av1_ec.h)."""
    from selkies_gstreamer_amd.ops.native import hip_device_count
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    L = _lib()
    P = ctypes.POINTER
    L.sk_av1_ec_tokens_cpu.argtypes = [P(ctypes.c_uint32), ctypes.c_int, ctypes.c_int, P(ctypes.c_uint8), ctypes.c_int]
    L.sk_av1_ec_tokens_cpu.restype = ctypes.c_int
    L.sk_av1_ec_tokens_hip.argtypes = [P(ctypes.c_uint32), P(ctypes.c_int32), P(ctypes.c_int32), ctypes.c_int,
                                       ctypes.c_int, P(ctypes.c_uint8), ctypes.c_int, P(ctypes.c_int32),
                                       P(ctypes.c_uint32)]
    L.sk_av1_cdf_words_cpu.argtypes = [P(ctypes.c_uint32), ctypes.c_int, ctypes.c_int, P(ctypes.c_uint32)]
    L.sk_av1_cdf_words_cpu.restype = ctypes.c_int
    L.sk_av1_ec_tokens_hip.restype = ctypes.c_int
    for qidx in (10, 100, 200):
        streams = _token_streams(L, qidx, 24)
        flat, offs, ns = [], [], []
        for s in streams:
            offs.append(len(flat))
            ns.append(len(s))
            flat += s
        cap = 8 * len(flat) + 4096
        out = np.zeros(cap, np.uint8)
        sizes = np.zeros(len(streams), np.int32)
        words = np.zeros(max(1, len(flat)), np.uint32)
        a32 = lambda x, t=ctypes.c_int32: (t * max(1, len(x)))(*x)   # noqa: E731
        rc = L.sk_av1_ec_tokens_hip(a32(flat, ctypes.c_uint32), a32(offs), a32(ns), len(streams), qidx,
                                    out.ctypes.data_as(P(ctypes.c_uint8)), cap, sizes.ctypes.data_as(P(ctypes.c_int32)),
                                    words.ctypes.data_as(P(ctypes.c_uint32)))
        assert rc == 0
        for t, s in enumerate(streams):   # phase A (k_av1_cdf) first: interval words
            ref = np.zeros(max(1, len(s)), np.uint32)
            L.sk_av1_cdf_words_cpu(a32(s, ctypes.c_uint32), len(s), qidx, ref.ctypes.data_as(P(ctypes.c_uint32)))
            got = words[offs[t]:offs[t] + len(s)]
            bad = np.nonzero(got != ref[:len(s)])[0]
            assert bad.size == 0, (qidx, t, bad[:5], got[bad[:5]], ref[bad[:5]])
        pos = 0
        for t, s in enumerate(streams):
            ref = (ctypes.c_uint8 * (8 * len(s) + 64))()
            m = L.sk_av1_ec_tokens_cpu(a32(s, ctypes.c_uint32), len(s), qidx, ref, len(ref))
            assert sizes[t] == m, (qidx, t)
            assert bytes(out[pos:pos + m]) == bytes(ref[:m]), (qidx, t)
            pos += m
