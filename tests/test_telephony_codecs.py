"""G.711 / G.722 (csrc/codec/telephony.cpp) and the WebRTC codec registry.

G.711 is pinned to the ITU-T G.711 code points (0 -> 0xFF u-law / 0xD5 A-law,
full scale -> 0x80/0x00 and 0xAA/0x2A) and checked exhaustively: every code word
decodes to a value that re-encodes to itself. G.722 has no reference decoder in
this image (parity unpinned against libavcodec): the ADPCM + QMF round trip must
reproduce tones with the SNR a 64 kbit/s G.722 reaches, after the QMF pair's
group delay.
"""
import numpy as np
import pytest

from selkies_gstreamer_amd.webrtc import codecs
from selkies_gstreamer_amd.webrtc.codecs import G711Decoder, G711Encoder, G722Decoder, G722Encoder


@pytest.mark.parametrize("alaw,zero,pmax,nmax", [(False, 0xFF, 0x80, 0x00), (True, 0xD5, 0xAA, 0x2A)])
def test_g711_code_points(alaw, zero, pmax, nmax):
    e = G711Encoder(alaw)
    assert e.encode(np.array([0, 32767, -32768], np.int16)) == bytes([zero, pmax, nmax])


@pytest.mark.parametrize("alaw", [False, True])
def test_g711_every_code_roundtrips(alaw):
    codes = bytes(range(256))
    pcm = G711Decoder(alaw).decode(codes)
    again = G711Encoder(alaw).encode(pcm)
    # u-law has two zeros (0x7F / 0xFF): both decode to 0, which encodes as 0xFF
    diff = [c for c, d in zip(codes, again) if c != d]
    assert diff == ([0x7F] if not alaw else [])


@pytest.mark.parametrize("alaw", [False, True])
def test_g711_sine_snr(alaw):
    t = np.arange(8000)
    x = (12000 * np.sin(2 * np.pi * 440 * t / 8000)).astype(np.int16)
    y = G711Decoder(alaw).decode(G711Encoder(alaw).encode(x))
    snr = 10 * np.log10(np.sum(x.astype(float) ** 2) / np.sum((x.astype(float) - y) ** 2))
    assert snr > 33


def _snr_aligned(x, y, max_delay=64):
    best = -1e9
    for d in range(max_delay):
        a, b = x[: len(x) - d].astype(float), y[d:].astype(float)
        a, b = a[200:], b[200:]   # skip adaptation start-up
        best = max(best, 10 * np.log10(np.sum(a ** 2) / max(1e-9, np.sum((a - b) ** 2))))
    return best


@pytest.mark.parametrize("freq,amp", [(440, 8000), (1000, 12000), (3000, 6000), (6000, 4000)])
def test_g722_tone_roundtrip(freq, amp):
    t = np.arange(16000)
    x = (amp * np.sin(2 * np.pi * freq * t / 16000)).astype(np.int16)
    enc, dec = G722Encoder(), G722Decoder()
    payload = b"".join(enc.encode(x[i:i + 320]) for i in range(0, len(x), 320))   # 20 ms packets
    assert len(payload) == len(x) // 2                     # 64 kbit/s
    y = np.concatenate([dec.decode(payload[i:i + 160]) for i in range(0, len(payload), 160)])
    assert len(y) == len(x)
    assert _snr_aligned(x, y) > 20


def test_g722_silence_stays_quiet_and_state_is_per_instance():
    enc1, enc2 = G722Encoder(), G722Encoder()
    z = np.zeros(640, np.int16)
    assert enc1.encode(z) == enc2.encode(z)
    y = G722Decoder().decode(enc1.encode(z))
    assert np.abs(y).max() < 64


def test_registry():
    assert codecs.find_codec("audio", "pcmu").payload_type == 0
    assert codecs.find_codec("audio", "G722").rtpmap == "G722/8000"
    assert codecs.find_codec("audio", "opus").rtpmap == "opus/48000/2"
    assert isinstance(codecs.get_encoder(codecs.find_codec("audio", "PCMA")), G711Encoder)
    with pytest.raises(KeyError):
        codecs.find_codec("video", "VP9")
