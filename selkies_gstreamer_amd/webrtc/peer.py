"""PeerConnection: ICE + DTLS-SRTP + SCTP data channels + RTP media on one
bundled UDP 5-tuple (RFC 8829 JSEP, RFC 8843 BUNDLE, rtcp-mux).

This is the server side of the reference's WebRTC mode — webrtcbin in
legacy/gstwebrtc_app.py (send-only H.264 + Opus, an "input" data channel,
keyframe on PLI/FIR, NACK retransmission, REMB-driven bitrate) and the
vendored aiortc RTCPeerConnection (webrtc/rtcpeerconnection.py). It also
implements the receiving side so the full stack is testable end to end
without a browser (tests/test_webrtc.py): a jitter buffer per SSRC
(webrtc/jitterbuffer.py), NACK on gaps, PLI on resets, and the delay-based
GCC estimator (webrtc/rate.py) that reports REMB to the sender.

Media plane per access unit: one native call packetises + SRTP-protects every
RTP packet (csrc/rtc/rtc.cpp); Python only hands the datagrams to the socket
and keeps a retransmission history.
"""
from __future__ import annotations

import asyncio
import logging
import random
import struct
import time
from typing import Callable, Optional

from . import rtp, sdp
from .fec import FecDecoder, FecEncoder
from .ice import Candidate, IceAgent
from .jitterbuffer import JitterBuffer, RtpPacket as JbPacket
from .rate import RemoteBitrateEstimator
from .native import Dtls, RtpPacketizer, Srtp
from .sctp import SctpAssociation, DataChannel

log = logging.getLogger("webrtc.peer")

HISTORY = 2048


class PeerConnection:
    def __init__(self, *, ice_lite: bool = False, addresses: Optional[list[str]] = None, port: int = 0,
                 stun_server: Optional[tuple] = None, video: bool = True, audio: bool = True, data: bool = True,
                 mtu: int = 1200, video_codec: str = "H264", turn_server: Optional[tuple] = None,
                 relay_only: bool = False, fec_percentage: int = 0, playout_delay_ms: Optional[tuple] = (0, 0)):
        self.ice_lite = ice_lite
        self._ice_args = dict(addresses=addresses, port=port, stun_server=stun_server, turn_server=turn_server,
                              relay_only=relay_only)
        self.want = dict(video=video, audio=audio, data=data)
        self.mtu = mtu
        self.ice: Optional[IceAgent] = None
        self.dtls: Optional[Dtls] = None
        self.sctp: Optional[SctpAssociation] = None
        self.srtp_tx: Optional[Srtp] = None
        self.srtp_rx: Optional[Srtp] = None
        self.local_sdp: Optional[sdp.SessionDescription] = None
        self.remote_sdp: Optional[sdp.SessionDescription] = None
        self.is_offerer = False
        self.dtls_role = "server"
        self.state = "new"
        self.video_ssrc = random.getrandbits(32) or 1
        self.audio_ssrc = random.getrandbits(32) or 2
        vc = video_codec.upper()
        self.video_codec = "H265" if vc in ("H265", "HEVC") else ("AV1" if vc == "AV1" else "H264")
        self._vpt = {"H265": sdp.H265_PT, "AV1": sdp.AV1_PT}.get(self.video_codec, sdp.H264_PT)
        self._vpk = RtpPacketizer(self.video_ssrc, self._vpt, mtu - 10, random.getrandbits(16))
        self._apk = RtpPacketizer(self.audio_ssrc, sdp.OPUS_PT, mtu - 10, random.getrandbits(16))
        self._history: dict[int, bytes] = {}
        self.fec_percentage = fec_percentage      # offered when > 0; active once the answer keeps RED
        self.playout_delay_ms = playout_delay_ms  # (min, max) ms; None: extension not offered
        self._fec_tx: Optional[FecEncoder] = None
        self._fec_rx = FecDecoder()
        self._sent = {"video_packets": 0, "video_bytes": 0, "audio_packets": 0, "audio_bytes": 0,
                      "retransmits": 0, "keyframe_requests": 0}
        self._last_ts = {self.video_ssrc: 0, self.audio_ssrc: 0}
        self._dtls_timer: Optional[asyncio.TimerHandle] = None
        self._dtls_done = asyncio.Event()
        self._tasks: list = []
        self._pending_channels: list = []
        # receive side
        self._depack: dict = {}   # ssrc -> H264Depacketizer / H265Depacketizer
        self._jitter: dict[int, JitterBuffer] = {}
        self._rx_rate: dict[int, RemoteBitrateEstimator] = {}
        self.remb_sent_bps: Optional[int] = None
        self._rx_seq: dict[int, int] = {}
        self.rtt_ms: Optional[float] = None
        self.remb_bps: Optional[int] = None
        # callbacks
        self.on_state: Callable[[str], None] = lambda st: None
        self.on_datachannel: Callable[[DataChannel], None] = lambda ch: None
        self.on_keyframe_request: Callable[[], None] = lambda: None
        self.on_bitrate: Callable[[int], None] = lambda bps: None
        self.on_video_frame: Callable[[bytes, int], None] = lambda au, ts: None
        self.on_audio_packet: Callable[[bytes, int], None] = lambda payload, ts: None
        self.on_ice_candidate: Callable[[Optional[Candidate]], None] = lambda c: None

    # -- negotiation --------------------------------------------------------------------------
    async def _gather(self, controlling: bool) -> None:
        if self.ice is None:
            self.ice = IceAgent(controlling=controlling, lite=self.ice_lite, **self._ice_args)
            self.ice.on_packet = self._on_packet
            self.ice.on_state = self._on_ice_state
            await self.ice.gather()
            for c in self.ice.local_candidates:
                self.on_ice_candidate(c)
            self.on_ice_candidate(None)

    async def create_offer(self) -> str:
        self.is_offerer = True
        await self._gather(controlling=True)
        self.dtls = Dtls("server")   # actpass: the answerer normally picks active
        self.local_sdp = sdp.build_offer(self.ice.local_ufrag, self.ice.local_pwd, self.dtls.fingerprint,
                                         self.ice.local_candidates, self.video_ssrc, self.audio_ssrc,
                                         ice_lite=self.ice_lite, video_codec=self.video_codec,
                                         fec=self.fec_percentage > 0, playout_delay=self.playout_delay_ms is not None,
                                         **self.want)
        return self.local_sdp.to_string()

    def _apply_negotiated(self) -> None:
        """After the answer: FEC only if the answer kept RED + ULPFEC, the playout-delay
        extension only if it kept the extmap (under the id it answered with)."""
        vid = next((m for m in self.remote_sdp.media if m.kind == "video"), None)
        if vid is None:
            return
        if self.fec_percentage > 0 and sdp.RED_PT in vid.fmts and sdp.ULPFEC_PT in vid.fmts:
            self._fec_tx = FecEncoder(self.video_ssrc, self.fec_percentage)
        eid = next((i for i, u in vid.extmap.items() if u == sdp.PLAYOUT_DELAY_URI), None)
        if eid is not None and self.playout_delay_ms is not None:
            self._vpk.set_playout_delay(eid, *self.playout_delay_ms)

    async def set_remote_description(self, text: str, kind: str) -> None:
        self.remote_sdp = sdp.parse(text)
        tr = self.remote_sdp.transport()
        if kind == "answer":
            if not self.is_offerer:
                raise ValueError("answer without a local offer")
            if tr["setup"] == "passive":   # the answerer wants to be the DTLS server
                self.dtls.set_role("client")
                self.dtls_role = "client"
            self._apply_negotiated()
        else:
            # an offer without an application section (e.g. the audio-only peer) gets no
            # SCTP association: the answerer would wait for one that never comes
            if not any(m.kind == "application" for m in self.remote_sdp.media):
                self.want["data"] = False
            # JSEP: the offerer controls unless it is ICE-lite
            await self._gather(controlling=self.remote_sdp.ice_lite)
        if tr["ufrag"] is None or tr["pwd"] is None or tr["fingerprint"] is None:
            raise ValueError("remote description lacks ICE credentials or a DTLS fingerprint")
        self.ice.set_remote_credentials(tr["ufrag"], tr["pwd"])
        if self.remote_sdp.ice_lite and self.ice.lite:
            raise ValueError("both sides are ICE-lite")
        if self.remote_sdp.ice_lite:
            self.ice.controlling = True
        self._remote_fp = tr["fingerprint"].split(None, 1)[-1]
        for c in tr["candidates"]:
            self.ice.add_remote_candidate(c)

    async def create_answer(self) -> str:
        if self.remote_sdp is None:
            raise ValueError("no remote offer")
        self.dtls = Dtls("client")   # setup:active
        self.dtls_role = "client"
        self.local_sdp = sdp.build_answer(self.remote_sdp, self.ice.local_ufrag, self.ice.local_pwd,
                                          self.dtls.fingerprint, self.ice.local_candidates, setup="active")
        return self.local_sdp.to_string()

    def add_ice_candidate(self, candidate: Optional[str]) -> None:
        if candidate:
            try:
                self.ice.add_remote_candidate(Candidate.from_sdp(candidate))
            except ValueError as e:
                log.debug("ignoring candidate: %s", e)
        else:
            self.ice.add_remote_candidate(None)

    # -- connection -----------------------------------------------------------------------------
    async def connect(self, timeout: float = 30.0) -> None:
        self._set_state("connecting")
        self.dtls.set_remote_fingerprint(self._remote_fp)
        try:
            await self.ice.connect(timeout)
            if self.dtls_role == "client":
                self._send_all(self.dtls.start())
                self._arm_dtls_timer()
            await asyncio.wait_for(self._dtls_done.wait(), timeout)
        except Exception:
            self._set_state("failed")
            raise
        if self.sctp is not None and self.sctp.is_client:
            await self.sctp.wait_established(timeout)
        self._set_state("connected")
        self._tasks.append(asyncio.ensure_future(self._rtcp_loop()))

    def _set_state(self, st: str) -> None:
        if st != self.state:
            self.state = st
            self.on_state(st)

    def _on_ice_state(self, st: str) -> None:
        if st in ("failed", "closed") and self.state not in ("closed",):
            self._set_state("failed" if st == "failed" else "closed")

    def _send_all(self, dgrams: list) -> None:
        for d in dgrams:
            self.ice.send(d)

    def _arm_dtls_timer(self) -> None:
        if self._dtls_timer:
            self._dtls_timer.cancel()
            self._dtls_timer = None
        ms = self.dtls.timeout_ms() if self.dtls else -1
        if ms >= 0:
            self._dtls_timer = asyncio.get_event_loop().call_later(max(ms, 1) / 1000.0, self._on_dtls_timer)

    def _on_dtls_timer(self) -> None:
        self._dtls_timer = None
        if self.dtls and self.dtls.state == Dtls.CONNECTING:
            self._send_all(self.dtls.on_timeout())
            self._arm_dtls_timer()

    def _on_packet(self, data: bytes, addr) -> None:
        b0 = data[0]
        if 20 <= b0 <= 63:
            self._on_dtls(data)
        elif 128 <= b0 <= 191 and self.srtp_rx is not None:
            if rtp.is_rtcp(data):
                pt = self.srtp_rx.unprotect_rtcp(data)
                if pt is not None:
                    self._on_rtcp(pt)
            else:
                pt = self.srtp_rx.unprotect_rtp(data)
                if pt is not None:
                    self._on_rtp(pt)

    def _on_dtls(self, data: bytes) -> None:
        try:
            done = self.dtls.feed(data)
        except Exception as e:
            log.error("DTLS failed: %s", e)
            self._set_state("failed")
            self._dtls_done.set()
            return
        self._send_all(self.dtls.pop())
        if done:
            local, remote = self.dtls.srtp_keys()
            self.srtp_tx, self.srtp_rx = Srtp(local), Srtp(remote)
            if self.want["data"]:
                self.sctp = SctpAssociation(self._sctp_send, is_client=self.dtls_role == "client")
                self.sctp.on_datachannel = self._on_remote_channel
                self.sctp.on_established = self._on_sctp_established
                self.sctp.start()
            self._dtls_done.set()
        else:
            self._arm_dtls_timer()
        if self.sctp is not None:
            for rec in self.dtls.read():
                self.sctp.feed(rec)

    def _sctp_send(self, packet: bytes) -> None:
        if self.dtls and self.dtls.state == Dtls.CONNECTED:
            self._send_all(self.dtls.write(packet))

    def _on_sctp_established(self) -> None:
        for ch in self._pending_channels:
            self._open_channel(ch)
        self._pending_channels.clear()

    def _on_remote_channel(self, ch: DataChannel) -> None:
        self.on_datachannel(ch)

    # -- data channels ----------------------------------------------------------------------------
    def create_data_channel(self, label: str, ordered: bool = True) -> "_ChannelHandle":
        h = _ChannelHandle(label, ordered)
        if self.sctp is not None and self.sctp.state == "established":
            self._open_channel(h)
        else:
            self._pending_channels.append(h)
        return h

    def _open_channel(self, h: "_ChannelHandle") -> None:
        ch = self.sctp.create_channel(h.label, h.ordered)
        h._bind(ch)

    # -- media send -------------------------------------------------------------------------------
    def send_video(self, annexb: bytes, timestamp: int) -> int:
        """Sends one H.264 / H.265 access unit (Annex-B) or AV1 temporal unit (OBUs) with a
        90 kHz timestamp."""
        if self.srtp_tx is None:
            return 0
        pack = {"H265": self._vpk.h265, "AV1": self._vpk.av1}.get(self.video_codec, self._vpk.h264)
        if self._fec_tx is None:
            pkts = pack(annexb, timestamp, self.srtp_tx)
        else:   # RED + ULPFEC over the plaintext packets, then SRTP
            plain = pack(annexb, timestamp, None)
            red = self._fec_tx.protect(plain, self._vpk.params.seq)
            self._vpk.params.seq = (self._vpk.params.seq + len(red) - len(plain)) & 0xFFFF
            pkts = [self.srtp_tx.protect_rtp(p) for p in red]
        for p in pkts:
            self.ice.send(p)
            self._history[struct.unpack_from("!H", p, 2)[0]] = p
        while len(self._history) > HISTORY:
            self._history.pop(next(iter(self._history)))
        self._sent["video_packets"] += len(pkts)
        self._sent["video_bytes"] += len(annexb)
        self._last_ts[self.video_ssrc] = timestamp
        return len(pkts)

    def send_audio(self, payload: bytes, timestamp: int) -> None:
        if self.srtp_tx is None:
            return
        self.ice.send(self._apk.raw(payload, timestamp, marker=False, srtp=self.srtp_tx))
        self._sent["audio_packets"] += 1
        self._sent["audio_bytes"] += len(payload)
        self._last_ts[self.audio_ssrc] = timestamp

    # -- RTCP -------------------------------------------------------------------------------------
    def _on_rtcp(self, data: bytes) -> None:
        fb = rtp.parse_rtcp(data)
        if self.video_ssrc in fb.pli:
            self._sent["keyframe_requests"] += 1
            self.on_keyframe_request()
        for media, lost in fb.nacks.items():
            if media != self.video_ssrc:
                continue
            for seq in lost:
                p = self._history.get(seq)
                if p is not None:
                    self.ice.send(p)
                    self._sent["retransmits"] += 1
        if fb.remb_bps is not None:
            self.remb_bps = fb.remb_bps
            self.on_bitrate(fb.remb_bps)
        for ssrc, _fl, _cum, _hs, _jit, lsr, dlsr in fb.reports:
            if ssrc == self.video_ssrc and lsr:
                hi, lo = rtp.ntp_now()
                now_mid = ((hi & 0xFFFF) << 16) | (lo >> 16)
                rtt = ((now_mid - lsr - dlsr) & 0xFFFFFFFF) / 65536.0
                if rtt < 60:
                    self.rtt_ms = rtt * 1000.0

    async def _rtcp_loop(self) -> None:
        while self.state == "connected":
            await asyncio.sleep(1.0)
            if self.srtp_tx is None:
                continue
            if self._sent["video_packets"]:
                sr = rtp.sender_report(self.video_ssrc, self._last_ts[self.video_ssrc], self._sent["video_packets"],
                                       self._sent["video_bytes"])
                self.ice.send(self.srtp_tx.protect_rtcp(sr))
            if self._sent["audio_packets"]:
                sr = rtp.sender_report(self.audio_ssrc, self._last_ts[self.audio_ssrc], self._sent["audio_packets"],
                                       self._sent["audio_bytes"])
                self.ice.send(self.srtp_tx.protect_rtcp(sr))

    def send_rtcp(self, packet: bytes) -> None:
        if self.srtp_tx is not None:
            self.ice.send(self.srtp_tx.protect_rtcp(packet))

    def request_keyframe(self, media_ssrc: int) -> None:
        """Receiver side: PLI towards the sender of media_ssrc."""
        self.send_rtcp(rtp.pli(self.video_ssrc, media_ssrc))

    # -- media receive (test peer / browser-less clients) -----------------------------------------------
    def _on_rtp(self, data: bytes) -> None:
        if len(data) >= 12 and data[1] & 0x7F == sdp.RED_PT:
            media, fec_seq = self._fec_rx.push(data)
            if fec_seq is not None:   # the FEC packet's seq is no loss: a filler for NACK / jitter buffer
                ssrc = struct.unpack_from("!I", data, 8)[0]
                self._track_seq(ssrc, fec_seq)
                jb = self._jitter.setdefault(ssrc, JitterBuffer(capacity=1024))
                jb.add(JbPacket(fec_seq, struct.unpack_from("!I", data, 4)[0], False, None))
            for pkt in media:         # unwrapped media, plus FEC-recovered packets
                self._on_rtp_media(pkt)
            return
        self._on_rtp_media(data)

    def _track_seq(self, ssrc: int, seq: int) -> None:
        exp = self._rx_seq.get(ssrc)
        if exp is not None and seq != exp and 0 < ((seq - exp) & 0xFFFF) < 64:
            lost = [(exp + i) & 0xFFFF for i in range((seq - exp) & 0xFFFF)]
            self.send_rtcp(rtp.nack(self.video_ssrc, ssrc, lost))
        if exp is None or 0 <= ((seq - exp) & 0xFFFF) < 0x8000:
            self._rx_seq[ssrc] = (seq + 1) & 0xFFFF

    def _on_rtp_media(self, data: bytes) -> None:
        h = rtp.parse_rtp(data)
        if h is None:
            return
        self._track_seq(h.ssrc, h.seq)
        payload = data[h.header_len:]
        if h.payload_type in (sdp.H264_PT, sdp.H265_PT, sdp.AV1_PT):
            now_ms = time.monotonic() * 1000.0
            est = self._rx_rate.setdefault(h.ssrc, RemoteBitrateEstimator())
            r = est.add(now_ms, h.timestamp / 90.0, len(data))
            if r is not None and r[1]:
                self.remb_sent_bps = r[0]
                self.send_rtcp(rtp.remb(self.video_ssrc, r[0], [h.ssrc]))
            jb = self._jitter.setdefault(h.ssrc, JitterBuffer(capacity=1024))
            pli, frames = jb.add(JbPacket(h.seq, h.timestamp, h.marker, payload))
            if pli:
                self.request_keyframe(h.ssrc)
            d = self._depack.get(h.ssrc)
            if d is None:
                d = self._depack[h.ssrc] = {sdp.H265_PT: rtp.H265Depacketizer,
                                            sdp.AV1_PT: rtp.AV1Depacketizer}.get(h.payload_type,
                                                                                rtp.H264Depacketizer)()
            for fr in frames:
                au = None
                for i, pk in enumerate(fr.packets):
                    au = d.push(pk.payload, fr.timestamp, pk.marker or i == len(fr.packets) - 1)
                if au:
                    self.on_video_frame(au, fr.timestamp)
        else:
            self.on_audio_packet(payload, h.timestamp)

    # -- stats / teardown ---------------------------------------------------------------------------
    def stats(self) -> dict:
        s = dict(self._sent)
        s.update({"state": self.state, "rtt_ms": self.rtt_ms, "remb_bps": self.remb_bps,
                  "ice_pair": self.ice.selected if self.ice else None, "dtls_role": self.dtls_role})
        if self.sctp is not None:
            s["sctp"] = dict(self.sctp.stats)
        return s

    async def close(self) -> None:
        self._set_state("closed")
        for t in self._tasks:
            t.cancel()
        if self._dtls_timer:
            self._dtls_timer.cancel()
        if self.sctp is not None:
            self.sctp.close()
        if self.dtls is not None and self.ice is not None:
            self._send_all(self.dtls.close())
        if self.ice is not None:
            await self.ice.close()


class _ChannelHandle:
    """A data channel created before the SCTP association is up."""

    def __init__(self, label: str, ordered: bool):
        self.label, self.ordered = label, ordered
        self.channel: Optional[DataChannel] = None
        self.on_message: Callable[[object], None] = lambda m: None
        self.on_open: Callable[[], None] = lambda: None
        self.on_close: Callable[[], None] = lambda: None
        self._open = asyncio.Event()

    def _bind(self, ch: DataChannel) -> None:
        self.channel = ch
        ch.on_message = lambda m: self.on_message(m)
        ch.on_close = lambda: self.on_close()

        def opened():
            self._open.set()
            self.on_open()
        ch.on_open = opened

    @property
    def ready_state(self) -> str:
        return self.channel.ready_state if self.channel else "connecting"

    async def wait_open(self, timeout: float = 10.0) -> None:
        await asyncio.wait_for(self._open.wait(), timeout)

    def send(self, data) -> None:
        if self.channel is None:
            raise ConnectionError("data channel not open yet")
        self.channel.send(data)

    def close(self) -> None:
        if self.channel:
            self.channel.close()
