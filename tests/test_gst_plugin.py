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
    for e in ("hiph264enc", "hiph265enc", "hipav1enc", "hipconvert", "hipupload", "hipdownload", "hipximagesrc"):
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
    assert len(outs[0]) == len(outs[1]) > 0
    # samples only: the rows' 4-byte padding of GstVideoInfo's layout is left unwritten
    w, h = W + 2, H + 1
    cw, ch = (w + 1) // 2, (h + 1) // 2
    ys, cs = (w + 3) & ~3, (cw + 3) & ~3
    fsz = ys * 2 * ch + 2 * cs * ch

    def visible(raw):
        fr = np.frombuffer(raw, np.uint8).reshape(-1, fsz)
        y = fr[:, : ys * h].reshape(-1, h, ys)[..., :w]
        c = fr[:, ys * 2 * ch:].reshape(-1, 2, ch, cs)[..., :cw]
        return y, c
    (ya, ca), (yb, cb) = visible(outs[0]), visible(outs[1])
    assert np.array_equal(ya, yb) and np.array_equal(ca, cb)


def test_reference_launch_string_runs_in_gstreamer(plugin, tmp_path):
    """legacy/pipeline.py run_gst: the reference's x264enc description (gstwebrtc_app.py:
    620-640 properties) runs in real GStreamer with hiph264enc in its place."""
    from selkies_gstreamer_amd.legacy import pipeline
    out = tmp_path / "ref.h264"
    text = (f"videotestsrc num-buffers=6 pattern=ball ! video/x-raw,format=BGRx,width={W},height={H},framerate=60/1 "
            "! cudaupload ! x264enc bitrate=2000 key-int-max=2147483647 speed-preset=ultrafast tune=zerolatency "
            f"! filesink location={out}")
    args = pipeline.to_gst_launch(text)
    assert "hiph264enc" in args and "hipupload" in args and "cudaupload" not in args and "bitrate=2000" in args
    r = pipeline.run_gst(text, timeout=300)
    assert r.returncode == 0, r.stderr
    assert len(_decode("h264", out.read_bytes())) == 6
    with pytest.raises(pipeline.PipelineError):
        pipeline.to_gst_launch("videotestsrc ! x264enc ! rtph264pay ! webrtcbin")


# ---------------------------------------------------------------------------------
# The reference's own graph topologies (legacy/gstwebrtc_app.py), videotestsrc in place
# of ximagesrc: a conversion and a format capsfilter always sit in front of the encoder.

def _nv12_planes(raw: bytes, w: int, h: int, n: int):
    """NV12 frames of a GstVideoInfo layout (4-byte row alignment) -> [(y, uv)]."""
    ys, cw, ch = (w + 3) & ~3, (w + 1) // 2, (h + 1) // 2
    uvs = (2 * cw + 3) & ~3
    fsize = ys * h + uvs * ch
    a = np.frombuffer(raw, np.uint8)
    assert a.size == n * fsize
    out = []
    for i in range(n):
        f = a[i * fsize:(i + 1) * fsize]
        out.append((f[:ys * h].reshape(h, ys)[:, :w], f[ys * h:].reshape(ch, uvs)[:, :2 * cw]))
    return out


def _i420_planes(raw: bytes, w: int, h: int, n: int):
    ys, cw, ch = (w + 3) & ~3, (w + 1) // 2, (h + 1) // 2
    cs = (cw + 3) & ~3
    fsize = ys * ((h + 1) & ~1) + 2 * cs * ch
    a = np.frombuffer(raw, np.uint8)
    assert a.size == n * fsize
    out = []
    for i in range(n):
        f = a[i * fsize:(i + 1) * fsize]
        uo = ys * ((h + 1) & ~1)
        out.append((f[:ys * h].reshape(h, ys)[:, :w], f[uo:uo + cs * ch].reshape(ch, cs)[:, :cw],
                    f[uo + cs * ch:uo + 2 * cs * ch].reshape(ch, cs)[:, :cw]))
    return out


def _planar_chain(tmp_path, codec, fmt, backend, w=W, h=H):
    """videotestsrc ! videoconvert ! video/x-raw,format=<fmt> ! tee -> raw planes + encoder."""
    raw, out = tmp_path / f"raw.{fmt}", tmp_path / f"out.{codec}"
    _launch(["videotestsrc", f"num-buffers={N}", "pattern=ball", "!",
             f"video/x-raw,format=BGRx,width={w},height={h},framerate=30/1", "!", "videoconvert", "!",
             f"video/x-raw,format={fmt}", "!", "tee", "name=t",
             "t.", "!", "queue", "!", "filesink", f"location={raw}",
             "t.", "!", "queue", "!", ENC[codec], f"backend={backend}", "!", "filesink", f"location={out}"])
    planes = (_nv12_planes if fmt == "NV12" else _i420_planes)(raw.read_bytes(), w, h, N)
    return planes, out.read_bytes()


def _native_planar(planes, codec, fmt, backend, w=W, h=H):
    from selkies_gstreamer_amd.ops.native import H264Encoder
    enc = H264Encoder(w, h, fullframe=True, codec=codec, backend=backend, qp=25, paint_qp=25, use_paint_over=False,
                      fps=30.0, rate_control="crf")
    out = b"".join(p.data[10:] for t, pl in enumerate(planes)
                   for p in enc.encode_yuv(fmt.lower(), *[np.ascontiguousarray(x) for x in pl], frame_id=t))
    enc.close()
    return out


@pytest.mark.parametrize("codec,fmt", [("h264", "NV12"), ("hevc", "I420"), ("av1", "I420")])
def test_reference_planar_chains_cpu(plugin, tmp_path, codec, fmt):
    """`videoconvert ! video/x-raw,format=NV12 ! x264enc` (gstwebrtc_app.py:611-617),
    `... format=I420 ! x265enc` (:667-683) and `... format=I420 ! svtav1enc` (:724-730)
    with the hip encoders in place: the element takes the planes GStreamer's own
    videoconvert made, its stream equals the native encoder fed the same planes, and an
    independent decoder returns them."""
    planes, stream = _planar_chain(tmp_path, codec, fmt, "cpu")
    assert stream == _native_planar(planes, codec, fmt, "cpu")
    ys = _decode(codec, stream)
    assert len(ys) == N
    for pl, y in zip(planes, ys):
        assert _psnr(y, pl[0]) > 30


def test_reference_launch_strings_with_capsfilters(plugin, tmp_path):
    """The reference's literal chains through legacy/pipeline.py (to_gst_launch maps the
    element names), run in real GStreamer: x264enc after `videoconvert ! NV12`, and the
    nvh264enc chain `cudaupload ! cudaconvert ! video/x-raw(memory:CUDAMemory),format=NV12`
    (-> hipupload ! hipconvert ! memory:HIPMemory caps, system memory on hosts without a
    HIP device)."""
    from selkies_gstreamer_amd.legacy import pipeline
    src = f"videotestsrc num-buffers={N} pattern=ball ! video/x-raw,format=BGRx,width={W},height={H},framerate=60/1"
    chains = {
        "x264": (f"{src} ! videoconvert ! video/x-raw,format=NV12 ! x264enc bitrate=2000 speed-preset=ultrafast "
                 "tune=zerolatency key-int-max=2147483647", "h264"),
        "nvh264": (f"{src} ! cudaupload ! cudaconvert ! video/x-raw(memory:CUDAMemory),format=NV12 ! nvh264enc "
                   "bitrate=2000 rc-mode=cbr gop-size=-1", "h264"),
        "x265": (f"{src} ! videoconvert ! video/x-raw,format=I420 ! x265enc bitrate=2000 speed-preset=ultrafast "
                 "tune=zerolatency key-int-max=2147483647", "hevc"),
        "svtav1": (f"{src} ! videoconvert ! video/x-raw,format=I420 ! svtav1enc target-bitrate=2000 preset=10",
                   "av1"),
    }
    for name, (text, codec) in chains.items():
        out = tmp_path / f"{name}.bin"
        args = pipeline.to_gst_launch(f"{text} ! filesink location={out}")
        if name == "nvh264":
            assert "hipupload" in args and "hipconvert" in args and "nvh264enc" not in args
        r = pipeline.run_gst(f"{text} ! filesink location={out}", timeout=300)
        assert r.returncode == 0, (name, r.stderr[-1500:])
        assert len(_decode(codec, out.read_bytes())) == N, name


def test_hipconvert_feeds_encoder_cpu(plugin, tmp_path):
    """`hipconvert ! hiph264enc` links (it could not in round 4): NV12 from the converter's
    K1 arithmetic gives the same stream as the encoder's own fused BGRx conversion."""
    raw, out = tmp_path / "raw.bgrx", tmp_path / "out.h264"
    _launch(["videotestsrc", f"num-buffers={N}", "pattern=ball", "!",
             f"video/x-raw,format=BGRx,width={W},height={H},framerate=30/1", "!", "tee", "name=t",
             "t.", "!", "queue", "!", "filesink", f"location={raw}",
             "t.", "!", "queue", "!", "hipconvert", "backend=cpu", "!", "hiph264enc", "backend=cpu", "!",
             "filesink", f"location={out}"])
    frames = np.fromfile(raw, np.uint8).reshape(N, H, W, 4)
    assert out.read_bytes() == _native(frames, "h264", "cpu")


def test_hipximagesrc_synthetic_cpu(plugin, tmp_path):
    """hipximagesrc (ximagesrc's properties; source=synthetic-* on hosts without X):
    region from startx/endx, paced at the negotiated framerate, its frames encode to the
    native encoder's stream."""
    raw, out = tmp_path / "raw.bgrx", tmp_path / "out.h264"
    w, h = 256, 128
    _launch(["hipximagesrc", "source=synthetic-motion", "startx=0", "starty=0", f"endx={w - 1}", f"endy={h - 1}",
             f"num-buffers={N}", "use-damage=true", "!", "video/x-raw,framerate=120/1", "!", "tee", "name=t",
             "t.", "!", "queue", "!", "filesink", f"location={raw}",
             "t.", "!", "queue", "!", "hiph264enc", "backend=cpu", "!", "filesink", f"location={out}"])
    frames = np.fromfile(raw, np.uint8).reshape(N, h, w, 4)
    assert len({f.tobytes() for f in frames}) > 1   # the synthetic desktop moves
    from selkies_gstreamer_amd.ops.native import H264Encoder
    enc = H264Encoder(w, h, fullframe=True, backend="cpu", qp=25, paint_qp=25, use_paint_over=False, fps=120.0,
                      rate_control="crf")
    ref = b"".join(p.data[10:] for t, f in enumerate(frames) for p in enc.encode(np.ascontiguousarray(f), t))
    assert out.read_bytes() == ref
    r = subprocess.run([build_gst.gst_bin("gst-launch-1.0"), "-q", "hipximagesrc", "display-name=:97", "num-buffers=1",
                        "!", "fakesink"], env=build_gst.gst_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "X display" in r.stderr   # no X server: a clear error, no crash


@pytest.mark.gpu
@pytest.mark.parametrize("codec,fmt", [("h264", "NV12"), ("hevc", "I420"), ("av1", "NV12")])
def test_reference_planar_chains_hip(plugin, tmp_path, codec, fmt):
    from selkies_gstreamer_amd.ops.native import hip_device_count
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    planes, stream = _planar_chain(tmp_path, codec, fmt, "hip")
    assert stream == _native_planar(planes, codec, fmt, "cpu")
    assert len(_decode(codec, stream)) == N


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["h264", "hevc", "av1"])
def test_hip_memory_chain(plugin, tmp_path, codec):
    """`hipupload ! hipconvert ! video/x-raw(memory:HIPMemory),format=NV12 ! hip*enc`: the
    frame crosses PCIe once and stays on the GPU through conversion and encoding (the
    reference's cudaupload / cudaconvert / nvh264enc chain). Same stream as the encoder's
    own BGRx path on the same frames."""
    from selkies_gstreamer_amd.ops.native import hip_device_count
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    raw, out = tmp_path / "raw.bgrx", tmp_path / f"out.{codec}"
    _launch(["videotestsrc", f"num-buffers={N}", "pattern=ball", "!",
             f"video/x-raw,format=BGRx,width={W},height={H},framerate=30/1", "!", "tee", "name=t",
             "t.", "!", "queue", "!", "filesink", f"location={raw}",
             "t.", "!", "queue", "!", "hipupload", "!", "hipconvert", "!",
             "video/x-raw(memory:HIPMemory),format=NV12", "!", ENC[codec], "backend=hip", "!",
             "filesink", f"location={out}"])
    frames = np.fromfile(raw, np.uint8).reshape(N, H, W, 4)
    assert out.read_bytes() == _native(frames, codec, "cpu")


@pytest.mark.gpu
def test_hip_upload_download_roundtrip(plugin, tmp_path):
    from selkies_gstreamer_amd.ops.native import hip_device_count
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    for fmt in ("BGRx", "I420", "NV12"):
        a, b = tmp_path / f"a.{fmt}", tmp_path / f"b.{fmt}"
        _launch(["videotestsrc", "num-buffers=3", "pattern=smpte", "!",
                 f"video/x-raw,format={fmt},width={W + 2},height={H + 1},framerate=30/1", "!", "tee", "name=t",
                 "t.", "!", "queue", "!", "filesink", f"location={a}",
                 "t.", "!", "queue", "!", "hipupload", "!", "video/x-raw(memory:HIPMemory)", "!", "hipdownload", "!",
                 "filesink", f"location={b}"])
        assert a.read_bytes() == b.read_bytes() and a.stat().st_size > 0, fmt
