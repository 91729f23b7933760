"""H.265 over RTP (RFC 7798): the native packetiser's single-NAL / aggregation /
fragmentation payloads reassemble to the original access unit, the SDP offer
carries H265/90000 on PT 100 (reference rtph265pay pt=100), and the legacy
pipeline front end maps the H.265 GStreamer encoder names onto the HIP HEVC encoder."""
import struct

from selkies_gstreamer_amd.legacy.pipeline import parse_pipeline
from selkies_gstreamer_amd.models.hevc.decoder import HevcDecoder, split_annexb
from selkies_gstreamer_amd.ops.native import HevcEncoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
from selkies_gstreamer_amd.webrtc import sdp
from selkies_gstreamer_amd.webrtc.native import RtpPacketizer
from selkies_gstreamer_amd.webrtc.rtp import H265Depacketizer, parse_rtp


def test_h265_packetize_roundtrip_and_decode():
    W, H = 320, 192
    enc = HevcEncoder(W, H, backend="cpu")
    src = SyntheticDesktop(W, H, kind="noise")
    pk = RtpPacketizer(0x1234, sdp.H265_PT, mtu=1200)
    dep = H265Depacketizer()
    dec = HevcDecoder()
    for t in range(3):
        au = enc.encode(src.frame(t), t)[0].data[10:]
        pkts = pk.h265(au, 3000 * t)
        assert all(len(p) <= 1200 for p in pkts)
        types = [(p[12] >> 1) & 63 for p in pkts]
        if t == 0:
            assert 48 in types            # VPS/SPS/PPS aggregated
        assert 49 in types                # large slices fragmented
        out = None
        for i, p in enumerate(pkts):
            h = parse_rtp(p)
            assert h.payload_type == sdp.H265_PT and h.timestamp == 3000 * t
            assert h.marker == (i == len(pkts) - 1)
            out = dep.push(p[h.header_len:], h.timestamp, h.marker)
        assert split_annexb(out) == split_annexb(au)
        assert len(dec.decode(out)) == 1
    enc.close()


def test_h265_offer_and_pipeline_mapping():
    off = sdp.build_offer("u", "p", "AA:BB", [], 1, 2, video_codec="H265")
    txt = off.to_string()
    assert "a=rtpmap:100 H265/90000" in txt and "profile-id=1" in txt
    spec = parse_pipeline("ximagesrc ! video/x-raw,framerate=60/1 ! x265enc bitrate=8000 ! rtph265pay mtu=1200 "
                          "! webrtcbin")
    assert spec.encoder == "h265" and spec.encoder_element == "x265enc" and spec.bitrate_kbps == 8000
