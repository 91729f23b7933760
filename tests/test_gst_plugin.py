"""GStreamer elements of libgsthip (csrc/gst/gsthip.c) inside real GStreamer 1.14 pipelines
(the /opt/conda install in this image; SURVEY §2.2, the reference's media graph in
legacy/gstwebrtc_app.py:200-1001).

Each pipeline tees the raw BGRx frames of ``videotestsrc`` to a file next to the
encoded stream, so the element's output can be checked two ways:
* byte for byte against the native encoder (ops.native, same settings) fed the same frames;
* decoded by an independent decoder (H.264 / HEVC: models/*/decoder.py, AV1: dav1d),
  close to the source frames.
hipconvert is checked against the BT.709 limited-range arithmetic in numpy.
CPU tier: backend=cpu; GPU tier (gpu-marked): backend=hip, same checks."""
import subprocess

import numpy as np
import pytest

from selkies_gstreamer_amd.ops import build_gst

pytestmark = pytest.mark.skipif(not build_gst.available(), reason="no GStreamer under " + str(build_gst.PREFIX))

W, H, N = 320, 192, 8
ENC = {"h264": "hiph264enc", "hevc": "hiph265enc", "av1": "hipav1enc"}


@pytest.fixture(scope="module")
def plugin():
    return build_gst.build()


def _launch(args, timeout=300):
    r = subprocess.run([build_gst.gst_bin("gst-launch-1.0"), "-q", *args], env=build_gst.gst_env(),
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]


def _encode(tmp_path, codec, backend, extra=()):
    raw, out = tmp_path / "raw.bgrx", tmp_path / f"out.{codec}"
    _launch(["videotestsrc", f"num-buffers={N}", "pattern=ball", "!",
             f"video/x-raw,format=BGRx,width={W},height={H},framerate=30/1", "!", "tee", "name=t",
             "t.", "!", "queue", "!", "filesink", f"location={raw}",
             "t.", "!", "queue", "!", ENC[codec], f"backend={backend}", *extra, "!", "filesink", f"location={out}"])
    frames = np.fromfile(raw, np.uint8).reshape(N, H, W, 4)
    return frames, out.read_bytes()


def _native(frames, codec, backend, **kw):
    from selkies_gstreamer_amd.ops.native import H264Encoder
    enc = H264Encoder(W, H, fullframe=True, codec=codec, backend=backend, qp=25, paint_qp=25, use_paint_over=False,
                      fps=30.0, rate_control=kw.pop("rate_control", "crf"), **kw)
    out = b"".join(p.data[10:] for t, f in enumerate(frames) for p in enc.encode(np.ascontiguousarray(f), t))
    enc.close()
    return out


def _obu_temporal_units(data: bytes) -> list:
    """Split a low-overhead AV1 stream at its temporal-delimiter OBUs."""
    tus, i, start = [], 0, 0
    while i < len(data):
        hdr = data[i]
        typ, ext = (hdr >> 3) & 15, (hdr >> 2) & 1
        j = i + 1 + ext
        size, shift = 0, 0
        while True:
            b = data[j]
            j += 1
            size |= (b & 127) << shift
            shift += 7
            if not b & 128:
                break
        if typ == 2 and i > start:
            tus.append(data[start:i])
            start = i
        i = j + size
    tus.append(data[start:])
    return tus


def _luma(f):
    r, g, b = (f[..., c].astype(np.int64) for c in (2, 1, 0))
    return ((47 * r + 157 * g + 16 * b + 128) >> 8) + 16


def _psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 99.0 if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


def _decode(codec, data):
    if codec == "h264":
        from selkies_gstreamer_amd.models.h264.decoder import H264Decoder
        return [p[0] for p in H264Decoder().decode(data)]
    if codec == "hevc":
        from selkies_gstreamer_amd.models.hevc.decoder import HevcDecoder
        return [p[0] for p in HevcDecoder().decode(data)]
    from selkies_gstreamer_amd.models.av1 import dav1d
    if not dav1d.available():
        pytest.skip("dav1d not available")
    dec = dav1d.Decoder()
    pics = [dec.decode(tu) for tu in _obu_temporal_units(data)]
    dec.close()
    return [p[0] for p in pics if p is not None]


def _check(tmp_path, codec, backend):
    frames, stream = _encode(tmp_path, codec, backend)
    assert stream == _native(frames, codec, backend), "element output differs from the native encoder"
    ys = _decode(codec, stream)
    assert len(ys) == N
    for f, y in zip(frames, ys):
        assert y.shape == (H, W)
        assert _psnr(y, _luma(f)) > 30


def test_inspect_lists_elements(plugin):
    r = subprocess.run([build_gst.gst_bin("gst-inspect-1.0"), "hip"], env=build_gst.gst_env(), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    for e in ("hiph264enc", "hiph265enc", "hipav1enc", "hipconvert"):
        assert e in r.stdout


@pytest.mark.parametrize("codec", ["h264", "hevc", "av1"])
def test_encoder_element_cpu(plugin, tmp_path, codec):
    _check(tmp_path, codec, "cpu")


def test_cbr_and_key_interval_cpu(plugin, tmp_path):
    """bitrate -> CBR (rate-control follows it), key-int-max -> a key frame every 4 frames."""
    frames, stream = _encode(tmp_path, "h264", "cpu", ["bitrate=600", "key-int-max=4"])
    from selkies_gstreamer_amd.models.h264.decoder import split_annexb
    idr = [n for n in split_annexb(stream) if n[0] & 31 == 5]
    sps = [n for n in split_annexb(stream) if n[0] & 31 == 7]
    assert len(sps) == 2 and len(idr) >= 2   # frames 0 and 4 (slices of one picture share the SPS)
    assert len(_decode("h264", stream)) == N


def test_hipconvert_cpu(plugin, tmp_path):
    raw, out = tmp_path / "raw.bgrx", tmp_path / "out.i420"
    _launch(["videotestsrc", "num-buffers=2", "pattern=smpte", "!",
             f"video/x-raw,format=BGRx,width={W + 2},height={H + 1},framerate=30/1", "!", "tee", "name=t",
             "t.", "!", "queue", "!", "filesink", f"location={raw}",
             "t.", "!", "queue", "!", "hipconvert", "backend=cpu", "!", "video/x-raw,format=I420", "!",
             "filesink", f"location={out}"])
    w, h = W + 2, H + 1
    f = np.fromfile(raw, np.uint8).reshape(2, h, w, 4)[0].astype(np.int64)
    cw, ch = (w + 1) // 2, (h + 1) // 2
    # GstVideoInfo I420 layout: rows padded to 4 bytes, the Y plane to an even height
    ys, cs = (w + 3) & ~3, (cw + 3) & ~3
    o = np.fromfile(out, np.uint8)
    frame = o[: o.size // 2]
    Y = frame[: ys * h].reshape(h, ys)[:, :w]
    uo = ys * 2 * ch
    U = frame[uo: uo + cs * ch].reshape(ch, cs)[:, :cw]
    assert np.array_equal(Y, np.clip(_luma(f), 0, 255))
    b, g, r = (np.pad(f[..., c], ((0, 2 * ch - h), (0, 2 * cw - w)), mode="edge") for c in (0, 1, 2))
    s = lambda x: x[0::2, 0::2] + x[0::2, 1::2] + x[1::2, 0::2] + x[1::2, 1::2]   # noqa: E731
    u = ((-26 * s(r) - 86 * s(g) + 112 * s(b) + 512) >> 10) + 128
    assert np.array_equal(U, np.clip(u, 0, 255))


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["h264", "hevc", "av1"])
def test_encoder_element_hip(plugin, tmp_path, codec):
    from selkies_gstreamer_amd.ops.native import hip_device_count
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    _check(tmp_path, codec, "hip")


@pytest.mark.gpu
def test_hipconvert_hip_matches_cpu(plugin, tmp_path):
    from selkies_gstreamer_amd.ops.native import hip_device_count
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    outs = []
    for be in ("cpu", "hip"):
        out = tmp_path / f"{be}.i420"
        _launch(["videotestsrc", "num-buffers=3", "pattern=ball", "!",
                 f"video/x-raw,format=BGRx,width={W + 2},height={H + 1},framerate=30/1", "!",
                 "hipconvert", f"backend={be}", "!", "video/x-raw,format=I420", "!", "filesink", f"location={out}"])
        outs.append(out.read_bytes())
    assert outs[0] == outs[1] and len(outs[0]) > 0


def test_reference_launch_string_runs_in_gstreamer(plugin, tmp_path):
    """legacy/pipeline.py run_gst: the reference's x264enc description (gstwebrtc_app.py:
    620-640 properties) runs in real GStreamer with hiph264enc in its place."""
    from selkies_gstreamer_amd.legacy import pipeline
    out = tmp_path / "ref.h264"
    text = (f"videotestsrc num-buffers=6 pattern=ball ! video/x-raw,format=BGRx,width={W},height={H},framerate=60/1 "
            "! cudaupload ! x264enc bitrate=2000 key-int-max=2147483647 speed-preset=ultrafast tune=zerolatency "
            f"! filesink location={out}")
    args = pipeline.to_gst_launch(text)
    assert "hiph264enc" in args and "cudaupload" not in args and "bitrate=2000" in args
    r = pipeline.run_gst(text, timeout=300)
    assert r.returncode == 0, r.stderr
    assert len(_decode("h264", out.read_bytes())) == 6
    with pytest.raises(pipeline.PipelineError):
        pipeline.to_gst_launch("videotestsrc ! x264enc ! rtph264pay ! webrtcbin")
