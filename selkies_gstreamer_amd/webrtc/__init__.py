"""WebRTC transport for the legacy (GStreamer-mode) streaming path.

Layers: :mod:`.stun` / :mod:`.ice` (connectivity), :mod:`.native` (DTLS-SRTP,
SRTP, RTP packetisation in C++ — csrc/rtc), :mod:`.sctp` (data channels),
:mod:`.rtp` (RTCP feedback, depacketiser), :mod:`.sdp` (offer/answer),
:mod:`.jitterbuffer` and :mod:`.rate` (receive side: reordering, GCC/REMB),
:mod:`.codecs` (codec registry; G.711 / G.722 native), :mod:`.contrib`
(relay, recorder, player, blackhole) and :mod:`.peer` (the PeerConnection
that ties them together).
"""
from .peer import PeerConnection  # noqa: F401
