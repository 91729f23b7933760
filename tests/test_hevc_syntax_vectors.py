"""Hand-worked vectors for the HEVC syntax the CTB-32 coding quadtree introduced, checked
against the test decoder's rules (models/hevc/decoder.py), which every encoder stream in the
tests is decoded with. The expected values are worked from the H.265 (04/2013) text, not from
the encoders: split_cu_flag ctxInc (9.3.4.2.2), part_mode binarisation (Table 9-43, AMP off),
the intra MPM list and rem mode mapping (8.4.2), and the merge / AMVP candidate lists
(8.5.3.2.2-8.5.3.2.6) with a single reference picture."""
import types

from selkies_gstreamer_amd.models.hevc import decoder as D


def test_split_cu_flag_ctx_inc():
    # condTerm = available && CtDepth[nb] > cqtDepth, summed over left and above
    assert D.split_cu_ctx_inc(True, 1, True, 1, 0) == 2      # CTB level, both neighbours split
    assert D.split_cu_ctx_inc(True, 0, True, 2, 0) == 1
    assert D.split_cu_ctx_inc(False, 2, True, 0, 0) == 0     # left unavailable (slice / picture edge)
    assert D.split_cu_ctx_inc(True, 2, True, 1, 1) == 1      # CU16 level: only depth 2 (CU8) counts
    assert D.split_cu_ctx_inc(True, 1, True, 1, 1) == 0


def _bins(*b):
    it = iter(b)
    used = []

    def dec(ctx_inc):
        used.append(ctx_inc)
        return next(it)
    return dec, used


def test_part_mode_binarisation():
    # inter CU32 (log2CbSize 5 > MinCbLog2SizeY 3, amp_enabled_flag 0): 2Nx2N "1", 2NxN "01",
    # Nx2N "00"; bin 0 ctxInc 0, bin 1 ctxInc 1 (Table 9-41)
    for bins, part in (((1,), 0), ((0, 1), 1), ((0, 0), 2)):
        dec, used = _bins(*bins)
        assert D.part_mode_of_bins(dec, False, 5, 3, False) == part
        assert used == [0, 1][:len(bins)]
    # intra at the minimum CB size (8x8): 2Nx2N "1", NxN "0"
    dec, used = _bins(1)
    assert D.part_mode_of_bins(dec, True, 3, 3, False) == 0
    dec, used = _bins(0)
    assert D.part_mode_of_bins(dec, True, 3, 3, False) == 3 and used == [0]


def test_mpm_candidate_list():
    # candA == candB < 2: planar, DC, vertical
    assert D.mpm_list(0, 0) == [0, 1, 26]
    assert D.mpm_list(1, 1) == [0, 1, 26]
    # candA == candB >= 2: A, 2 + ((A + 29) % 32), 2 + ((A - 2 + 1) % 32)
    assert D.mpm_list(10, 10) == [10, 9, 11]
    assert D.mpm_list(2, 2) == [2, 33, 3]
    assert D.mpm_list(34, 34) == [34, 33, 3]
    # candA != candB: A, B, then planar unless one is planar, else DC unless one is DC, else 26
    assert D.mpm_list(10, 26) == [10, 26, 0]
    assert D.mpm_list(0, 26) == [0, 26, 1]
    assert D.mpm_list(1, 0) == [1, 0, 26]
    # rem_intra_luma_pred_mode: increment past each (ascending) candidate it reaches
    assert D.mode_from_rem(0, [10, 26, 0]) == 1
    assert D.mode_from_rem(8, [10, 26, 0]) == 9
    assert D.mode_from_rem(9, [10, 26, 0]) == 11
    assert D.mode_from_rem(31, [10, 26, 0]) == 34


def _fake(motion, max_merge=5):
    """A decoder stand-in whose neighbour at luma (x, y) has motion `motion[(x, y)]` (None or
    absent: unavailable or intra)."""
    f = types.SimpleNamespace(max_merge=max_merge)
    f._nb_motion = lambda x0, y0, xn, yn: motion.get((xn, yn))
    return f


def test_merge_candidates():
    # 16x16 PU at (16, 16): A1 (15, 31), B1 (31, 15), B0 (32, 15), A0 (15, 32), B2 (15, 15)
    m = {(15, 31): (4, 0), (31, 15): (4, 0), (32, 15): (8, 0), (15, 15): (4, 0)}
    # B1 pruned against A1, B0 kept (differs from B1), A0 unavailable, B2 pruned against A1;
    # then zero candidates (refIdx 0: the single reference) up to MaxNumMergeCand
    assert D.HevcDecoder._merge_cands(_fake(m), 16, 16, 16, 16) == [(4, 0), (8, 0), (0, 0), (0, 0), (0, 0)]
    m = {(15, 31): (1, 0), (31, 15): (2, 0), (32, 15): (3, 0), (15, 32): (4, 0), (15, 15): (5, 0)}
    # four spatial candidates available: B2 is not considered
    assert D.HevcDecoder._merge_cands(_fake(m), 16, 16, 16, 16) == [(1, 0), (2, 0), (3, 0), (4, 0), (0, 0)]
    # PART_2NxN, partIdx 1 of a 32x32 CU at (0, 0): the PU is (0, 16) 32x16; B1 (31, 15) lies in
    # PU 0 and is not a candidate; B0 (32, 15) is compared with B1 only when B1 is available
    m = {(-1, 31): (1, 1), (31, 15): (2, 2), (32, 15): (2, 2)}
    assert D.HevcDecoder._merge_cands(_fake(m), 0, 16, 32, 16, part=1, pidx=1)[:2] == [(1, 1), (2, 2)]
    # PART_Nx2N, partIdx 1: the PU is (16, 0) 16x32; A1 (15, 31) lies in PU 0
    m = {(15, 31): (7, 7), (31, -1): (3, 3)}
    assert D.HevcDecoder._merge_cands(_fake(m), 16, 0, 16, 32, part=2, pidx=1)[:2] == [(3, 3), (0, 0)]


def test_amvp_candidates():
    # A1 and B0 carry the same vector: one of them, then the zero candidate
    m = {(15, 31): (3, 0), (32, 15): (3, 0), (15, 15): (5, 5)}
    assert D.HevcDecoder._amvp_cands(_fake(m), 16, 16, 16, 16) == [(3, 0), (0, 0)]
    # no A candidate (isScaledFlag 0): mvA takes mvB (B0), mvB is re-derived from B0..B2 and
    # equals it, so it is removed
    m = {(32, 15): (2, 1), (31, 15): (9, 9)}
    assert D.HevcDecoder._amvp_cands(_fake(m), 16, 16, 16, 16) == [(2, 1), (0, 0)]
    # A0 first among A, B1 (B0 unavailable) for B
    m = {(15, 32): (1, 2), (15, 31): (6, 6), (31, 15): (4, 4)}
    assert D.HevcDecoder._amvp_cands(_fake(m), 16, 16, 16, 16) == [(1, 2), (4, 4)]
