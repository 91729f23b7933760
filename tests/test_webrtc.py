"""WebRTC transport (legacy WebRTC mode): STUN/ICE, DTLS-SRTP, SRTP vectors,
RTP packetisation, SCTP data channels and a full two-peer loopback over UDP.

Parity with a browser is checked against published vectors (RFC 5769 STUN,
RFC 3711 key derivation, the libsrtp AES-CM/HMAC-SHA1-80 packet vector);
interop with a live browser is "parity unpinned" (no browser in CI)."""
import asyncio
import os
import struct

import pytest

from selkies_gstreamer_amd.webrtc import rtp, sdp, stun
from selkies_gstreamer_amd.webrtc.native import Dtls, DtlsError, RtpPacketizer, Srtp, crc32c
from selkies_gstreamer_amd.webrtc.peer import PeerConnection
from selkies_gstreamer_amd.webrtc.sctp import SctpAssociation


def run(coro, timeout=30):
    return asyncio.run(asyncio.wait_for(coro, timeout))


def test_stun_rfc5769_request_vector():
    raw = bytes.fromhex(
        "000100582112a442b7e7a701bc34d686fa87dfae"
        "802200105354554e207465737420636c69656e74"
        "002400046e0001ff"
        "80290008932ff9b151263b36"
        "000600096576746a3a68367659202020"
        "000800149aeaa70cbfd8cb56781ef2b5b2d3f249c1b571a2"
        "80280004e57a3bcf")
    msg, offs = stun.decode(raw)
    assert msg.method == stun.BINDING and msg.cls == stun.REQUEST
    assert msg.attrs[stun.USERNAME] == "evtj:h6vY"
    assert msg.attrs[stun.PRIORITY] == 0x6E0001FF
    assert msg.attrs[stun.ICE_CONTROLLED] == 0x932FF9B151263B36
    assert stun.check_integrity(raw, offs, b"VOkJxbRl1RmTxUk/WvJxBt")
    assert not stun.check_integrity(raw, offs, b"wrong")
    assert stun.check_fingerprint(raw, offs)


def test_stun_encode_roundtrip_xor_address():
    m = stun.Message(stun.BINDING, stun.SUCCESS)
    m.attrs[stun.XOR_MAPPED_ADDRESS] = ("192.0.2.1", 32853)
    raw = m.encode(b"key")
    d, offs = stun.decode(raw)
    assert d.cls == stun.SUCCESS and d.attrs[stun.XOR_MAPPED_ADDRESS] == ("192.0.2.1", 32853)
    assert stun.check_integrity(raw, offs, b"key") and stun.check_fingerprint(raw, offs)


def test_srtp_rfc3711_and_libsrtp_vectors():
    s = Srtp(bytes.fromhex("E1F97A0D3E018BE0D64FA32C06DE4139" "0EC675AD498AFEEBB6960B3AABE6"))
    k = s.session_keys()
    assert k[:16].hex() == "c61e7a93744f39ee10734afe3ff7a087"               # RFC 3711 B.3 cipher key
    assert k[16:36].hex() == "cebe321f6ff7716b6fd4ab49af256a156d38baa4"     # auth key
    assert k[36:50].hex() == "30cbbc08863d8c85d49db34a9ae1"                 # cipher salt
    pt = bytes.fromhex("800f1234decafbadcafebabe" + "ab" * 16)
    ct = s.protect_rtp(pt)
    assert ct.hex() == ("800f1234decafbadcafebabe4e55dc4ce79978d88ca4d215949d2402"
                        "b78d6acc99ea179b8dbb")


def test_srtp_roundtrip_replay_and_tamper():
    key = os.urandom(30)
    tx, rx = Srtp(key), Srtp(key)
    for seq in (65534, 65535, 0, 1):   # across the ROC wrap
        pkt = struct.pack("!BBHII", 0x80, 97, seq, 1234, 0xABCD) + os.urandom(50)
        c = tx.protect_rtp(pkt)
        assert rx.unprotect_rtp(c) == pkt
        assert rx.unprotect_rtp(c) is None    # replay
    bad = bytearray(tx.protect_rtp(struct.pack("!BBHII", 0x80, 97, 2, 1, 0xABCD) + b"x" * 20))
    bad[15] ^= 1
    assert rx.unprotect_rtp(bytes(bad)) is None
    sr = rtp.sender_report(0xABCD, 9000, 10, 1000)
    c = tx.protect_rtcp(sr)
    assert rx.unprotect_rtcp(c) == sr


def test_crc32c_check_value():
    assert crc32c(b"123456789") == 0xE3069283
    assert crc32c(b"") == 0


def _payload(n):
    """Random NAL payload without zero bytes (no start-code emulation, non-zero last byte)."""
    return os.urandom(n).replace(b"\x00", b"\x01")


def test_h264_packetize_roundtrip():
    sps = b"\x67\x42\xe0\x1f" + _payload(8)
    pps = b"\x68\xce\x3c\x80"
    idr = b"\x65" + _payload(5000)
    small = b"\x41" + _payload(300)
    au = b"".join(b"\x00\x00\x00\x01" + n for n in (sps, pps, idr))
    pk = RtpPacketizer(0x1234, 97, mtu=1190, seq=65530)
    pkts = pk.h264(au, 90000)
    assert all(len(p) <= 1190 for p in pkts)
    assert (pkts[0][12] & 0x1F) == 24            # SPS+PPS aggregated (STAP-A)
    assert (pkts[1][12] & 0x1F) == 28            # IDR fragmented (FU-A)
    assert pkts[-1][1] & 0x80 and not any(p[1] & 0x80 for p in pkts[:-1])
    d = rtp.H264Depacketizer()
    out = [d.push(p[12:], 90000, bool(p[1] & 0x80)) for p in pkts]
    assert out[-1] == au and all(o is None for o in out[:-1])
    assert pk.seq == (65530 + len(pkts)) & 0xFFFF
    p2 = pk.h264(b"\x00\x00\x01" + small, 93000)
    assert len(p2) == 1 and d.push(p2[0][12:], 93000, True) == b"\x00\x00\x00\x01" + small


def test_rtcp_feedback_parsing():
    data = (rtp.pli(1, 42) + rtp.nack(1, 42, [100, 101, 105, 130]) + rtp.remb(1, 2_500_000, [42]) +
            rtp.fir(1, 43, 7) + rtp.receiver_report(1, 42, 12, 3, 70000, 5))
    fb = rtp.parse_rtcp(data)
    assert fb.pli == {42, 43}
    assert sorted(fb.nacks[42]) == [100, 101, 105, 130]
    assert abs(fb.remb_bps - 2_500_000) / 2_500_000 < 1e-4
    assert fb.reports[0][:4] == (42, 12, 3, 70000)


def test_sdp_offer_answer_roundtrip():
    from selkies_gstreamer_amd.webrtc.ice import Candidate
    cand = [Candidate("1", 1, "udp", 2130706431, "10.0.0.5", 40000, "host")]
    off = sdp.build_offer("abcd", "p" * 22, "AA:BB", cand, 11, 22)
    text = off.to_string()
    p = sdp.parse(text)
    assert [m.kind for m in p.media] == ["video", "audio", "application"]
    assert p.bundle == ["0", "1", "2"]
    v = p.media[0]
    assert v.rtpmap[97] == "H264/90000" and sdp.fmtp_params(v.fmtp[97])["packetization-mode"] == "1"
    assert "nack pli" in v.rtcp_fb[97] and v.direction == "sendonly" and v.ssrc == 11
    assert p.transport()["candidates"][0].port == 40000 and p.media[2].sctp_port == 5000
    ans = sdp.parse(sdp.build_answer(p, "wxyz", "q" * 22, "CC:DD", []).to_string())
    assert ans.media[0].direction == "recvonly" and ans.transport()["setup"] == "active"


def _pump(a, b, drop=lambda i, d: False):
    """Moves datagrams between two in-memory DTLS endpoints until both are idle."""
    i = 0
    qa, qb = [], []
    for _ in range(50):
        qa += a.pop()
        qb += b.pop()
        if not qa and not qb:
            return
        for d in qa:
            i += 1
            if not drop(i, d):
                b.feed(d)
        for d in qb:
            i += 1
            if not drop(i, d):
                a.feed(d)
        qa, qb = [], []


def test_dtls_srtp_handshake_in_memory():
    srv, cli = Dtls("server"), Dtls("client")
    srv.set_remote_fingerprint(cli.fingerprint)
    cli.set_remote_fingerprint(srv.fingerprint.lower())
    for d in cli.start():
        srv.feed(d)
    _pump(srv, cli)
    assert srv.state == Dtls.CONNECTED and cli.state == Dtls.CONNECTED
    sl, sr = srv.srtp_keys()
    cl, cr = cli.srtp_keys()
    assert sl == cr and sr == cl and sl != cl
    for d in cli.write(b"hello sctp"):
        srv.feed(d)
    assert srv.read() == [b"hello sctp"]


def test_dtls_rejects_wrong_fingerprint():
    srv, cli = Dtls("server"), Dtls("client")
    cli.set_remote_fingerprint("00:" * 31 + "00")
    for d in cli.start():
        srv.feed(d)
    with pytest.raises(DtlsError):
        _pump(srv, cli)


def _sctp_pair(loss=None):
    q = {"a": [], "b": []}
    a = SctpAssociation(lambda d: q["b"].append(d), is_client=True)
    b = SctpAssociation(lambda d: q["a"].append(d), is_client=False)
    n = [0]

    async def pump(rounds=200):
        for _ in range(rounds):
            moved = False
            for dst, key in ((a, "a"), (b, "b")):
                while q[key]:
                    d = q[key].pop(0)
                    n[0] += 1
                    moved = True
                    if loss and loss(n[0], d):
                        continue
                    dst.feed(d)
            await asyncio.sleep(0 if moved else 0.01)
    return a, b, pump


def test_sctp_datachannel_messages_and_fragmentation():
    async def main():
        a, b, pump = _sctp_pair()
        got, chans = [], []
        b.on_datachannel = lambda ch: (chans.append(ch), setattr(ch, "on_message", got.append))
        a.start()
        await pump(20)
        assert a.state == b.state == "established"
        ch = a.create_channel("input")
        await pump(20)
        assert ch.ready_state == "open" and chans[0].label == "input" and chans[0].id % 2 == 0
        big = os.urandom(70000)
        ch.send("kd,65")
        ch.send(big)
        ch.send("")
        await pump(50)
        assert got == ["kd,65", big, ""]
        back = []
        ch.on_message = back.append
        chans[0].send("pong")
        await pump(20)
        assert back == ["pong"]
        ch.close()
        await pump(20)
        assert chans[0].ready_state == "closed"
    run(main())


def test_sctp_retransmits_lost_data():
    async def main():
        drops = set()

        def loss(i, d):  # drop every 3rd packet once the association is up
            if i > 12 and i % 3 == 0 and i not in drops:
                drops.add(i)
                return True
            return False
        a, b, pump = _sctp_pair(loss)
        got = []
        b.on_datachannel = lambda ch: setattr(ch, "on_message", got.append)
        a.start()
        await pump(30)
        ch = a.create_channel("data")
        await pump(30)
        msgs = [os.urandom(2000 + i) for i in range(20)]
        for m in msgs:
            ch.send(m)
        for _ in range(40):
            await pump(10)
            if len(got) == len(msgs):
                break
            await asyncio.sleep(0.1)
        assert got == msgs
        assert a.stats["retransmits"] > 0
    run(main(), timeout=60)


@pytest.mark.parametrize("lite", [False, True])
def test_peer_connection_loopback(lite):
    """Offerer (server: H.264 + data channel) <-> answerer (viewer) over UDP on 127.0.0.1."""
    async def main():
        srv = PeerConnection(ice_lite=lite, addresses=["127.0.0.1"], audio=True)
        cli = PeerConnection(addresses=["127.0.0.1"])
        offer = await srv.create_offer()
        await cli.set_remote_description(offer, "offer")
        answer = await cli.create_answer()
        await srv.set_remote_description(answer, "answer")
        assert srv.dtls_role == "server" and cli.dtls_role == "client"

        frames, keyreq, dc_msgs, audio = [], [], [], []
        cli.on_video_frame = lambda au, ts: frames.append((au, ts))
        cli.on_audio_packet = lambda p, ts: audio.append(p)
        srv.on_keyframe_request = lambda: keyreq.append(1)
        cli_channels = []
        cli.on_datachannel = lambda ch: (cli_channels.append(ch), setattr(ch, "on_message", dc_msgs.append))
        await asyncio.gather(srv.connect(10), cli.connect(10))
        assert srv.state == cli.state == "connected"

        inp = srv.create_data_channel("input")
        await inp.wait_open(5)
        srv_in = []
        inp.on_message = srv_in.append
        inp.send('{"type":"stats"}')
        for _ in range(50):
            if cli_channels:
                break
            await asyncio.sleep(0.02)
        cli_channels[0].send("kd,65293")

        aus = [b"\x00\x00\x00\x01\x67\x42\xe0\x1f" + _payload(6) + b"\x00\x00\x00\x01\x68\xce\x3c\x80" +
               b"\x00\x00\x00\x01\x65" + _payload(20000)]
        aus += [b"\x00\x00\x00\x01\x41" + _payload(3000 + 100 * i) for i in range(5)]
        # lose one packet of the third frame: the viewer NACKs, the server retransmits from history
        orig = srv.ice.send
        state = {"n": 0}

        def lossy(d):
            if (d[1] & 0x7F) == sdp.H264_PT:
                state["n"] += 1
                if state["n"] == 20:
                    return
            orig(d)
        srv.ice.send = lossy
        for i, au in enumerate(aus):
            srv.send_video(au, 3000 * i)
            srv.send_audio(os.urandom(80), 960 * i)
            await asyncio.sleep(0.01)
        for _ in range(100):
            if len(frames) >= len(aus) - 1:
                break
            await asyncio.sleep(0.02)
        got = {ts: au for au, ts in frames}
        assert got[0] == aus[0] and got[3000 * 5] == aus[5]
        assert len(audio) == len(aus)
        assert srv.stats()["retransmits"] >= 1
        cli.request_keyframe(srv.video_ssrc)
        for _ in range(50):
            if keyreq and dc_msgs and srv_in:
                break
            await asyncio.sleep(0.02)
        assert keyreq and dc_msgs == ['{"type":"stats"}'] and srv_in == ["kd,65293"]
        await cli.close()
        await srv.close()
    run(main(), timeout=60)
