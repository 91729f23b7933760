"""Video FEC (RED + ULPFEC, webrtc/fec.py) and the playout-delay header extension
(native packetiser) — reference: gstwebrtc_app.py:996-1000 (fec-type ulp-red) and
PlayoutDelayExtension (1744-1780)."""
import asyncio
import os
import struct

import pytest

from selkies_gstreamer_amd.webrtc import rtp, sdp
from selkies_gstreamer_amd.webrtc.fec import FecDecoder, FecEncoder, red_unwrap, red_wrap
from selkies_gstreamer_amd.webrtc.native import RtpPacketizer
from selkies_gstreamer_amd.webrtc.peer import PeerConnection


def _au(n):
    # no zero bytes: random payload could otherwise hold a start code and split the NAL
    return b"\x00\x00\x00\x01\x65" + bytes(b | 1 for b in os.urandom(n))


def _seq(p):
    return struct.unpack_from("!H", p, 2)[0]


def test_red_roundtrip():
    pk = RtpPacketizer(0x1234, sdp.H264_PT, 1200, 100)
    for p in pk.h264(_au(3000), 9000):
        r = red_wrap(p)
        assert r[1] & 0x7F == sdp.RED_PT and r[1] & 0x80 == p[1] & 0x80
        assert red_unwrap(r) == p


@pytest.mark.parametrize("size,pct", [(20000, 25), (50000, 5), (900, 100)])
def test_ulpfec_recovers_one_loss_per_group(size, pct):
    pk = RtpPacketizer(0xABCD, sdp.H264_PT, 1200, 65530)   # sequence numbers wrap inside the unit
    media = pk.h264(_au(size), 123456)
    enc = FecEncoder(0xABCD, pct)
    out = enc.protect(media, pk.params.seq)
    n_fec = len(out) - len(media)
    assert n_fec >= 1 and [_seq(red_unwrap(p)) for p in out[len(media):]] == \
        [(pk.params.seq + i) & 0xFFFF for i in range(n_fec)]
    # drop the first media packet of every FEC group
    per = -(-len(media) // n_fec)
    lost = set(range(0, len(media), per))
    dec = FecDecoder()
    got = {}
    for i, p in enumerate(out):
        if i in lost:
            continue
        media_out, fec_seq = dec.push(p)
        assert (fec_seq is not None) == (i >= len(media))
        for m in media_out:
            got[_seq(m)] = m
    assert dec.recovered == len(lost)
    assert [got[_seq(m)] for m in media] == media   # byte-identical, marker bit included


def test_ulpfec_two_losses_in_a_group_are_not_recovered():
    pk = RtpPacketizer(1, sdp.H264_PT, 1200, 0)
    media = pk.h264(_au(8000), 0)
    out = FecEncoder(1, 10).protect(media, pk.params.seq)   # one FEC packet for the unit
    dec = FecDecoder()
    for i, p in enumerate(out):
        if i not in (1, 2):
            dec.push(p)
    assert dec.recovered == 0


@pytest.mark.parametrize("mn,mx", [(0, 0), (100, 500)])
def test_playout_delay_extension(mn, mx):
    pk = RtpPacketizer(7, sdp.H264_PT, 1200, 0)
    pk.set_playout_delay(sdp.PLAYOUT_DELAY_ID, mn, mx)
    au = b"\x00\x00\x00\x01\x67\x42\xe0\x1f\x00\x00\x00\x01\x68\xce\x3c\x80" + _au(5000)
    pkts = pk.h264(au, 90000)
    d = rtp.H264Depacketizer()
    out = None
    for p in pkts:
        assert len(p) <= 1200
        assert p[0] & 0x10 and p[12:16] == b"\xbe\xde\x00\x01"
        assert p[16] == (sdp.PLAYOUT_DELAY_ID << 4) | 2
        assert ((p[17] << 4) | (p[18] >> 4), ((p[18] & 15) << 8) | p[19]) == (mn // 10, mx // 10)
        h = rtp.parse_rtp(p)
        assert h.header_len == 20
        out = d.push(p[h.header_len:], h.timestamp, h.marker)
    assert out == au


def test_sdp_offers_red_ulpfec_and_playout_delay():
    off = sdp.build_offer("u", "p" * 22, "AA:" * 31 + "AA", [], 1, 2, fec=True)
    text = off.to_string()
    assert "a=rtpmap:123 red/90000" in text and "a=rtpmap:125 ulpfec/90000" in text
    assert f"a=extmap:{sdp.PLAYOUT_DELAY_ID} {sdp.PLAYOUT_DELAY_URI}" in text
    back = sdp.parse(text)
    assert back.media[0].extmap == {sdp.PLAYOUT_DELAY_ID: sdp.PLAYOUT_DELAY_URI}
    assert back.media[0].fmts == [sdp.H264_PT, sdp.RED_PT, sdp.ULPFEC_PT]


def test_peer_fec_recovers_losses_without_retransmission():
    """Offerer with 30 % FEC and playout delay; the viewer's NACKs are ignored by the
    sender (history disabled), so every lost packet must come back through ULPFEC."""
    async def main():
        srv = PeerConnection(addresses=["127.0.0.1"], audio=False, data=False, fec_percentage=30,
                             playout_delay_ms=(0, 0))
        cli = PeerConnection(addresses=["127.0.0.1"], audio=False, data=False)
        offer = await srv.create_offer()
        await cli.set_remote_description(offer, "offer")
        await srv.set_remote_description(await cli.create_answer(), "answer")
        assert srv._fec_tx is not None and srv._vpk.params.playout_ext_id == sdp.PLAYOUT_DELAY_ID
        frames = []
        cli.on_video_frame = lambda au, ts: frames.append((au, ts))
        await asyncio.gather(srv.connect(10), cli.connect(10))
        srv._history.clear()
        orig = srv.ice.send
        count = {"n": 0}

        fec_seqs = set()
        protect = srv._fec_tx.protect

        def recording_protect(media, next_seq):
            out = protect(media, next_seq)
            fec_seqs.update(_seq(p) for p in out[len(media):])
            return out
        srv._fec_tx.protect = recording_protect

        def lossy(d):
            # SRTP encrypts the RED block header; the sequence number (clear) tells FEC from media
            if len(d) > 12 and d[1] & 0x7F == sdp.RED_PT and _seq(d) not in fec_seqs:
                count["n"] += 1
                if count["n"] % 9 == 3:   # 1 in 9 media packets lost (at most one per FEC group)
                    return
            orig(d)
        srv.ice.send = lossy
        send_video = srv.send_video

        def no_history(au, ts):
            n = send_video(au, ts)
            srv._history.clear()   # no retransmission: only FEC can repair
            return n
        aus = [_au(6000 + 500 * i) for i in range(8)]
        for i, au in enumerate(aus):
            no_history(au, 3000 * i)
            await asyncio.sleep(0.01)
        for _ in range(500):   # up to 10 s: the CPU tier runs with -n workers competing for cores
            if len(frames) >= len(aus):
                break
            await asyncio.sleep(0.02)
        got = {ts: au for au, ts in frames}
        assert cli._fec_rx.recovered >= 3
        assert [got.get(3000 * i) for i in range(len(aus))] == aus
        await cli.close()
        await srv.close()
    asyncio.run(asyncio.wait_for(main(), 60))
