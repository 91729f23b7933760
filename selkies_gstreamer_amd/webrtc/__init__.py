"""WebRTC transport for the legacy (GStreamer-mode) streaming path.

Layers: :mod:`.stun` / :mod:`.ice` (connectivity), :mod:`.native` (DTLS-SRTP,
SRTP, RTP packetisation in C++ — csrc/rtc), :mod:`.sctp` (data channels),
:mod:`.rtp` (RTCP feedback, depacketiser), :mod:`.sdp` (offer/answer) and
:mod:`.peer` (the PeerConnection that ties them together).
"""
from .peer import PeerConnection  # noqa: F401
