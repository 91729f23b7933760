"""SDP offer/answer for the streaming session (RFC 8866 / JSEP subset).

The server is the offerer, like the reference's webrtcbin pipeline
(legacy/gstwebrtc_app.py:808-1000, on-negotiation-needed → create-offer):
one BUNDLE group with a send-only H.264 video section (packetization-mode=1,
Constrained Baseline ``42e01f`` — what the HIP encoder emits; RTCP feedback
nack, nack pli, ccm fir, goog-remb), a send-only Opus section and the
``webrtc-datachannel`` application section for input/stats.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Optional

from .ice import Candidate

H264_PT = 97
H265_PT = 100   # reference: rtph265pay pt=100 (legacy/gstwebrtc_app.py:848-866)
AV1_PT = 96     # reference: rtpav1pay payload=96 (legacy/gstwebrtc_app.py:924-934)
OPUS_PT = 111
RED_PT = 123
ULPFEC_PT = 125
SCTP_PORT = 5000


@dataclass
class Media:
    kind: str                      # video / audio / application
    port: int = 9
    protocol: str = "UDP/TLS/RTP/SAVPF"
    fmts: list = field(default_factory=list)
    mid: str = ""
    direction: str = "sendrecv"
    rtpmap: dict = field(default_factory=dict)     # pt -> "H264/90000"
    fmtp: dict = field(default_factory=dict)       # pt -> "a=b;c=d"
    rtcp_fb: dict = field(default_factory=dict)    # pt -> ["nack", "nack pli", ...]
    ssrc: Optional[int] = None
    cname: str = ""
    msid: str = ""
    ice_ufrag: Optional[str] = None
    ice_pwd: Optional[str] = None
    fingerprint: Optional[str] = None              # "sha-256 AB:CD..."
    setup: Optional[str] = None
    candidates: list = field(default_factory=list)
    end_of_candidates: bool = False
    sctp_port: Optional[int] = None
    max_message_size: Optional[int] = None
    rtcp_mux: bool = False
    extmap: dict = field(default_factory=dict)     # id -> header extension URI (RFC 8285)


PLAYOUT_DELAY_URI = "http://www.webrtc.org/experiments/rtp-hdrext/playout-delay"
PLAYOUT_DELAY_ID = 6


@dataclass
class SessionDescription:
    media: list = field(default_factory=list)
    session_id: int = 0
    bundle: list = field(default_factory=list)
    ice_lite: bool = False
    ice_ufrag: Optional[str] = None
    ice_pwd: Optional[str] = None
    fingerprint: Optional[str] = None
    setup: Optional[str] = None

    # effective transport parameters (session level falls back to the first media)
    def transport(self) -> dict:
        m0 = self.media[0] if self.media else Media("")
        return {"ufrag": m0.ice_ufrag or self.ice_ufrag, "pwd": m0.ice_pwd or self.ice_pwd,
                "fingerprint": m0.fingerprint or self.fingerprint, "setup": m0.setup or self.setup,
                "candidates": [c for m in self.media for c in m.candidates]}

    def to_string(self) -> str:
        ln = ["v=0", f"o=- {self.session_id or int(time.time() * 1000)} 2 IN IP4 127.0.0.1", "s=-", "t=0 0"]
        if self.bundle:
            ln.append("a=group:BUNDLE " + " ".join(self.bundle))
        if self.ice_lite:
            ln.append("a=ice-lite")
        ln.append("a=msid-semantic: WMS *")
        for m in self.media:
            ln.append(f"m={m.kind} {m.port} {m.protocol} {' '.join(str(f) for f in m.fmts)}")
            ln.append("c=IN IP4 0.0.0.0")
            if m.kind != "application":
                ln.append("a=rtcp:9 IN IP4 0.0.0.0")
            for c in m.candidates:
                ln.append("a=candidate:" + c.to_sdp())
            if m.end_of_candidates:
                ln.append("a=end-of-candidates")
            if m.ice_ufrag:
                ln += [f"a=ice-ufrag:{m.ice_ufrag}", f"a=ice-pwd:{m.ice_pwd}", "a=ice-options:trickle"]
            if m.fingerprint:
                ln.append(f"a=fingerprint:{m.fingerprint}")
            if m.setup:
                ln.append(f"a=setup:{m.setup}")
            ln.append(f"a=mid:{m.mid}")
            if m.kind == "application":
                if m.sctp_port is not None:
                    ln.append(f"a=sctp-port:{m.sctp_port}")
                if m.max_message_size is not None:
                    ln.append(f"a=max-message-size:{m.max_message_size}")
                continue
            ln.append(f"a={m.direction}")
            if m.msid:
                ln.append(f"a=msid:{m.msid}")
            if m.rtcp_mux:
                ln.append("a=rtcp-mux")
            for eid, uri in sorted(m.extmap.items()):
                ln.append(f"a=extmap:{eid} {uri}")
            for pt in m.fmts:
                if pt in m.rtpmap:
                    ln.append(f"a=rtpmap:{pt} {m.rtpmap[pt]}")
                for fb in m.rtcp_fb.get(pt, []):
                    ln.append(f"a=rtcp-fb:{pt} {fb}")
                if pt in m.fmtp:
                    ln.append(f"a=fmtp:{pt} {m.fmtp[pt]}")
            if m.ssrc is not None:
                ln.append(f"a=ssrc:{m.ssrc} cname:{m.cname}")
                if m.msid:
                    ln.append(f"a=ssrc:{m.ssrc} msid:{m.msid}")
        return "\r\n".join(ln) + "\r\n"


def parse(text: str) -> SessionDescription:
    sd = SessionDescription()
    cur: Optional[Media] = None
    for raw in text.splitlines():
        line = raw.strip()
        if len(line) < 2 or line[1] != "=":
            continue
        k, v = line[0], line[2:]
        if k == "o":
            try:
                sd.session_id = int(v.split()[1])
            except (IndexError, ValueError):
                pass
        elif k == "m":
            b = v.split()
            fmts = [int(f) if f.isdigit() else f for f in b[3:]]
            cur = Media(b[0], int(b[1]), b[2], fmts)
            sd.media.append(cur)
        elif k == "a":
            name, _, val = v.partition(":")
            tgt = cur
            if name == "group" and val.startswith("BUNDLE"):
                sd.bundle = val.split()[1:]
            elif name == "ice-lite":
                sd.ice_lite = True
            elif name == "ice-ufrag":
                if tgt: tgt.ice_ufrag = val
                else: sd.ice_ufrag = val
            elif name == "ice-pwd":
                if tgt: tgt.ice_pwd = val
                else: sd.ice_pwd = val
            elif name == "fingerprint":
                if tgt: tgt.fingerprint = val
                else: sd.fingerprint = val
            elif name == "setup":
                if tgt: tgt.setup = val
                else: sd.setup = val
            elif tgt is None:
                continue
            elif name == "mid":
                tgt.mid = val
            elif name in ("sendrecv", "sendonly", "recvonly", "inactive"):
                tgt.direction = name
            elif name == "rtcp-mux":
                tgt.rtcp_mux = True
            elif name == "rtpmap":
                pt, _, enc = val.partition(" ")
                tgt.rtpmap[int(pt)] = enc
            elif name == "fmtp":
                pt, _, p = val.partition(" ")
                if pt.isdigit():
                    tgt.fmtp[int(pt)] = p
            elif name == "rtcp-fb":
                pt, _, fb = val.partition(" ")
                if pt.isdigit():
                    tgt.rtcp_fb.setdefault(int(pt), []).append(fb)
            elif name == "ssrc":
                ssrc, _, attr = val.partition(" ")
                if tgt.ssrc is None:
                    tgt.ssrc = int(ssrc)
                if attr.startswith("cname:"):
                    tgt.cname = attr[6:]
            elif name == "msid":
                tgt.msid = val
            elif name == "extmap":
                eid, _, uri = val.partition(" ")
                eid = eid.split("/")[0]
                if eid.isdigit():
                    tgt.extmap[int(eid)] = uri.split()[0] if uri else ""
            elif name == "candidate":
                try:
                    tgt.candidates.append(Candidate.from_sdp(val))
                except ValueError:
                    pass
            elif name == "end-of-candidates":
                tgt.end_of_candidates = True
            elif name == "sctp-port":
                tgt.sctp_port = int(val)
            elif name == "max-message-size":
                tgt.max_message_size = int(val)
            elif name == "sctpmap":  # legacy: a=sctpmap:5000 webrtc-datachannel 1024
                tgt.sctp_port = int(val.split()[0])
    return sd


def fmtp_params(s: str) -> dict:
    out = {}
    for kv in s.split(";"):
        k, _, v = kv.strip().partition("=")
        if k:
            out[k] = v
    return out


def h264_fmtp(profile_level_id: str = "42e01f") -> str:
    return f"level-asymmetry-allowed=1;packetization-mode=1;profile-level-id={profile_level_id}"


def h265_fmtp(level_id: int = 153) -> str:
    return f"level-id={level_id};profile-id=1;tier-flag=0;tx-mode=SRST"


def av1_fmtp(level_idx: int = 8) -> str:
    """AV1 RTP fmtp: Main profile, Main tier (level_idx 8 = 4.0; the sequence header
    carries the real level)."""
    return f"level-idx={level_idx};profile=0;tier=0"


def build_offer(ufrag: str, pwd: str, fingerprint: str, candidates: list, video_ssrc: int, audio_ssrc: int,
                video: bool = True, audio: bool = True, data: bool = True, cname: str = "selkies",
                ice_lite: bool = False, profile_level_id: str = "42e01f",
                video_codec: str = "H264", fec: bool = False, playout_delay: bool = True) -> SessionDescription:
    """fec: offer RED + ULPFEC next to the video codec (gstwebrtc_app.py:996-1000);
    playout_delay: offer the playout-delay header extension (PlayoutDelayExtension,
    gstwebrtc_app.py:1744-1780)."""
    sd = SessionDescription(session_id=int(time.time() * 1000), ice_lite=ice_lite)
    common = dict(ice_ufrag=ufrag, ice_pwd=pwd, fingerprint=f"sha-256 {fingerprint}", setup="actpass",
                  candidates=list(candidates), end_of_candidates=True)
    if video:
        if video_codec.upper() in ("H265", "HEVC"):
            pt, rtpmap, fmtp = H265_PT, "H265/90000", h265_fmtp()
        elif video_codec.upper() == "AV1":
            pt, rtpmap, fmtp = AV1_PT, "AV1/90000", av1_fmtp()
        else:
            pt, rtpmap, fmtp = H264_PT, "H264/90000", h264_fmtp(profile_level_id)
        fmts, rtpmaps = [pt], {pt: rtpmap}
        if fec:
            fmts += [RED_PT, ULPFEC_PT]
            rtpmaps.update({RED_PT: "red/90000", ULPFEC_PT: "ulpfec/90000"})
        sd.media.append(Media(
            "video", fmts=fmts, mid=str(len(sd.media)), direction="sendonly", rtcp_mux=True,
            rtpmap=rtpmaps, fmtp={pt: fmtp},
            rtcp_fb={pt: ["nack", "nack pli", "ccm fir", "goog-remb"]}, ssrc=video_ssrc, cname=cname,
            msid="selkies video0", extmap={PLAYOUT_DELAY_ID: PLAYOUT_DELAY_URI} if playout_delay else {},
            **common))
    if audio:
        sd.media.append(Media(
            "audio", fmts=[OPUS_PT], mid=str(len(sd.media)), direction="sendonly", rtcp_mux=True,
            rtpmap={OPUS_PT: "opus/48000/2"}, fmtp={OPUS_PT: "minptime=10;useinbandfec=1;stereo=1;sprop-stereo=1"},
            ssrc=audio_ssrc, cname=cname, msid="selkies audio0", **common))
    if data:
        sd.media.append(Media("application", protocol="UDP/DTLS/SCTP", fmts=["webrtc-datachannel"],
                              mid=str(len(sd.media)), sctp_port=SCTP_PORT, max_message_size=262144, **common))
    sd.bundle = [m.mid for m in sd.media]
    return sd


def build_answer(offer: SessionDescription, ufrag: str, pwd: str, fingerprint: str, candidates: list,
                 setup: str = "active") -> SessionDescription:
    """Answer accepting every offered section (used by the test peer and by
    browser-offer deployments); send-only sections are answered recvonly."""
    sd = SessionDescription(session_id=int(time.time() * 1000), bundle=list(offer.bundle))
    flip = {"sendonly": "recvonly", "recvonly": "sendonly", "sendrecv": "sendrecv", "inactive": "inactive"}
    for om in offer.media:
        m = Media(om.kind, protocol=om.protocol, fmts=list(om.fmts), mid=om.mid, direction=flip[om.direction],
                  rtpmap=dict(om.rtpmap), fmtp=dict(om.fmtp), rtcp_fb={k: list(v) for k, v in om.rtcp_fb.items()},
                  ice_ufrag=ufrag, ice_pwd=pwd, fingerprint=f"sha-256 {fingerprint}", setup=setup,
                  candidates=list(candidates), end_of_candidates=True, sctp_port=om.sctp_port,
                  max_message_size=om.max_message_size, rtcp_mux=om.rtcp_mux, extmap=dict(om.extmap))
        sd.media.append(m)
    return sd
