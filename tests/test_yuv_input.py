"""Planar 4:2:0 input (sk_h264_encode_yuv): the encoders take I420 / NV12 frames, as
the reference's GStreamer graphs deliver them to x264enc / x265enc / svtav1enc after a
`videoconvert ! video/x-raw,format=NV12|I420` capsfilter (legacy/gstwebrtc_app.py:
611-617, 667-683, 724-730), and device-resident planes (the `memory:HIPMemory` caps,
the analogue of nvh264enc's CUDAMemory input at :261-284).

Oracle: the encoders' own BGRx path. Converting a BGRx frame with the K1 arithmetic
(convert_bgrx = hipconvert's converter) and feeding the planes must give the BGRx
path's bitstream byte for byte at macroblock-aligned sizes (edge padding differs at
other sizes: planar input repeats the last chroma sample, K1 the last pixel pair)."""
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder, convert_bgrx
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
from tests.h264_util import StripeDecoder, bgrx_to_y709, psnr


def _kw(codec):
    return dict(codec=codec, fullframe=codec != "h264")


@pytest.mark.parametrize("codec", ["h264", "hevc", "av1"])
def test_planar_input_equals_bgrx_path_cpu(codec):
    W, H = 256, 128
    src = SyntheticDesktop(W, H, kind="motion")
    a, b, c = (H264Encoder(W, H, backend="cpu", **_kw(codec)) for _ in range(3))
    for t in range(4):
        f = src.frame(t)
        pa = a.encode(f, t)
        pb = b.encode_yuv("i420", *convert_bgrx(f, "i420"), frame_id=t)
        pc = c.encode_yuv("nv12", *convert_bgrx(f, "nv12"), frame_id=t)
        assert [p.data for p in pb] == [p.data for p in pa], (codec, t)
        assert [p.data for p in pc] == [p.data for p in pa], (codec, t)


def test_planar_input_odd_size_decodes_cpu():
    """Non-aligned sizes: the planar path pads by repeating the edge samples; the stream
    decodes to the input planes."""
    W, H = 200, 90
    src = SyntheticDesktop(W, H, kind="desktop")
    enc = H264Encoder(W, H, backend="cpu", stripe_height=32, qp=20)
    sd = StripeDecoder(W, H)
    for t in range(3):
        f = src.frame(t)
        y, u, v = convert_bgrx(f, "i420")
        for p in enc.encode_yuv("i420", y, u, v, frame_id=t):
            sd.feed(p.data)
        assert psnr(sd.Y, bgrx_to_y709(f)) > 35
    with pytest.raises(KeyError):
        enc.encode_yuv("yuy2", y, u, v)


def test_converter_nv12_matches_i420_cpu():
    f = SyntheticDesktop(130, 66, kind="noise").frame(0)
    y, u, v = convert_bgrx(f, "i420")
    y2, uv = convert_bgrx(f, "nv12")
    assert np.array_equal(y, y2)
    assert np.array_equal(uv[:, 0::2], u) and np.array_equal(uv[:, 1::2], v)


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["h264", "hevc", "av1"])
def test_planar_input_hip_matches_cpu(codec):
    """k_yuv_damage (HIP) == load_frame_yuv (CPU) for host planes and for device planes
    (DevicePlane: hipMalloc'd, the encoder reads them without a host copy)."""
    from selkies_gstreamer_amd.ops.native import DevicePlane, require_gpu
    require_gpu()
    W, H = 200, 90   # unaligned: exercises the padding rule
    src = SyntheticDesktop(W, H, kind="motion")
    cpu, hip_host, hip_dev = (H264Encoder(W, H, backend=b, **_kw(codec)) for b in ("cpu", "hip", "hip"))
    for t in range(5):
        f = src.frame(t)
        fmt = "nv12" if t % 2 else "i420"
        planes = convert_bgrx(f, fmt)
        pc = cpu.encode_yuv(fmt, *planes, frame_id=t)
        ph = hip_host.encode_yuv(fmt, *planes, frame_id=t)
        dev = [DevicePlane(p) for p in planes]
        pd = hip_dev.encode_yuv(fmt, *dev, frame_id=t)
        for d in dev:
            d.close()
        assert [p.data for p in ph] == [p.data for p in pc], (codec, t, "host planes")
        assert [p.data for p in pd] == [p.data for p in pc], (codec, t, "device planes")
    # back to BGRx on the same session: graphs re-captured with k_convert_damage
    f = src.frame(9)
    assert [p.data for p in hip_host.encode(f, 9)] == [p.data for p in cpu.encode(f, 9)]


@pytest.mark.gpu
def test_converter_hip_matches_cpu():
    from selkies_gstreamer_amd.ops.native import require_gpu
    require_gpu()
    f = SyntheticDesktop(322, 182, kind="noise").frame(0)
    for fmt in ("i420", "nv12"):
        a, b = convert_bgrx(f, fmt, backend="cpu"), convert_bgrx(f, fmt, backend="hip")
        assert all(np.array_equal(x, y) for x, y in zip(a, b)), fmt
