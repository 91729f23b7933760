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


@pytest.mark.gpu
def test_gpu_tiles_match_host_encoder():
    """k_av1_ec_tiles (csrc/kernels/av1_kernels.hip): 24 independent tiles coded on
    the GPU, each byte-identical to the host encoder and decodable by the spec model."""
    from selkies_gstreamer_amd.ops.native import hip_device_count
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    L = _lib()
    P = ctypes.POINTER
    L.sk_av1_ec_encode_tiles_hip.argtypes = [P(ctypes.c_uint32), P(ctypes.c_int32), P(ctypes.c_int32), ctypes.c_int,
                                             P(ctypes.c_uint16), P(ctypes.c_int32), ctypes.c_int, ctypes.c_int,
                                             P(ctypes.c_uint8), P(ctypes.c_int32)]
    L.sk_av1_ec_encode_tiles_hip.restype = ctypes.c_int
    rng = np.random.default_rng(11)
    nctx = 12
    nsym = [int(rng.integers(2, 17)) for _ in range(nctx)]
    cdfs = [_random_cdf(rng, n, 0.5) for n in nsym]
    tiles, words, offs, ns = 24, [], [], []
    for t in range(tiles):
        offs.append(len(words))
        n = int(rng.integers(0, 2500))
        ns.append(n)
        for _ in range(n):
            k = int(rng.choice([0, 0, 0, 1, 2]))
            if k == 0:
                c = int(rng.integers(nctx))
                words.append((c << 20) | int(rng.integers(nsym[c])))
            elif k == 1:
                words.append((1 << 30) | int(rng.integers(2)))
            else:
                b = int(rng.integers(1, 17))
                words.append((2 << 30) | (b << 20) | int(rng.integers(1 << b)))
    flat = np.zeros(nctx * 17, np.uint16)
    for c, cdf in enumerate(cdfs):
        flat[c * 17:c * 17 + len(cdf)] = cdf
    out = np.zeros(2 * len(words) + 8 * tiles, np.uint8)
    sizes = np.zeros(tiles, np.int32)
    a32 = lambda x, t=ctypes.c_int32: (t * len(x))(*x)   # noqa: E731
    rc = L.sk_av1_ec_encode_tiles_hip(a32(words, ctypes.c_uint32), a32(offs), a32(ns), tiles,
                                      flat.ctypes.data_as(P(ctypes.c_uint16)), a32(nsym), nctx, 1,
                                      out.ctypes.data_as(P(ctypes.c_uint8)), sizes.ctypes.data_as(P(ctypes.c_int32)))
    assert rc == 0
    for t in range(tiles):
        w = words[offs[t]:offs[t] + ns[t]]
        kind = [x >> 30 for x in w]
        ctx = [(x >> 20) & 1023 for x in w]
        sym = [x & 0xfffff for x in w]
        host = _encode(kind, ctx, sym, [list(c) for c in cdfs], nsym, True)
        base = 2 * offs[t] + 8 * t
        gpu = bytes(out[base:base + sizes[t]])
        assert gpu == host, t
