"""GStreamer pipeline-string front end for the legacy WebRTC mode.

The reference's legacy engine is a GStreamer graph (legacy/gstwebrtc_app.py:
``ximagesrc ! videoconvert ! x264enc ... ! rtph264pay ! webrtcbin`` and the
cuda*/va* variants). This build has no GStreamer: capture,
conversion and encoding are one fused HIP pipeline. So that deployments that
describe their media graph as a launch string keep working, this module parses
the same syntax and maps element names and properties onto the engine's
settings ("a minimal in-process pipeline string parser that maps
the same element names and properties to our engine").

Mapping:
* sources: ``ximagesrc`` (display-name, show-pointer, startx/starty/endx/endy,
  use-damage), ``videotestsrc`` / ``hipsrc`` → synthetic content;
* caps ``video/x-raw,width=..,height=..,framerate=N/D``;
* conversion / upload (``videoconvert``, ``cudaupload``, ``cudaconvert``,
  ``vapostproc``, ``hipupload``, ``hipconvert``, ``queue``) → fused into the HIP
  convert kernel (scaling is not: caps must keep the capture size);
* H.264 encoders (``x264enc``, ``nvh264enc``, ``vah264enc``, ``openh264enc``,
  ``qsvh264enc``, ``hiph264enc``) → the gfx950 H.264 encoder, H.265 encoders (``x265enc``,
  ``nvh265enc``, ``vah265enc``, ``qsvh265enc``, ``hiph265enc``) → the gfx950 HEVC encoder,
  AV1 encoders (``av1enc``, ``svtav1enc``, ``rav1enc``, ``nvav1enc``, ``vaav1enc``,
  ``qsvav1enc``, ``hipav1enc``) → the gfx950 AV1 encoder:
  ``bitrate`` / ``target-bitrate`` (kbit/s),
  ``key-int-max`` / ``gop-size`` / ``keyframe-period``, ``quantizer`` / ``qp-const``;
  ``jpegenc`` → the JPEG stripe encoder;
* payloaders ``rtph264pay`` / ``rtph265pay`` / ``rtpav1pay`` (``mtu``), ``webrtcbin`` (``stun-server``,
  ``latency``);
* audio ``pulsesrc`` (``device``) → ``opusenc`` (``bitrate``, ``frame-size``) →
  ``rtpopuspay``.
VP8 / VP9 encoder elements are rejected with an explicit error: this build's video
codecs are H.264, H.265, AV1 and JPEG.

When GStreamer itself is installed (the 1.14 under /opt/conda in this image) a launch
string can also run in real GStreamer: :func:`to_gst_launch` rewrites the reference's
encoder elements to this build's GStreamer elements (libgsthip, csrc/gst/: ``hiph264enc``
/ ``hiph265enc`` / ``hipav1enc``) with their properties mapped, ``ximagesrc`` to
``hipximagesrc``, ``cudaupload`` / ``cudaconvert`` / ``cudadownload`` to ``hipupload`` /
``hipconvert`` / ``hipdownload`` and ``memory:CUDAMemory`` caps to ``memory:HIPMemory``,
and :func:`run_gst` runs it with gst-launch-1.0. That covers graphs
GStreamer can complete here (file / fd / fake sinks); ``webrtcbin`` and the RTP
payloaders are not in that GStreamer build, so WebRTC stays on the own stack (webrtc/).
"""
from __future__ import annotations

import shlex
from dataclasses import dataclass, field
from typing import Optional

H264_ENCODERS = {"x264enc", "nvh264enc", "vah264enc", "vah264lpenc", "openh264enc", "qsvh264enc", "hiph264enc",
                 "nvcudah264enc", "nvautogpuh264enc"}
H265_ENCODERS = {"x265enc", "nvh265enc", "vah265enc", "vah265lpenc", "qsvh265enc", "hiph265enc", "nvcudah265enc",
                 "nvautogpuh265enc"}
AV1_ENCODERS = {"av1enc", "svtav1enc", "rav1enc", "nvav1enc", "vaav1enc", "qsvav1enc", "hipav1enc",
                "nvcudaav1enc"}
UNSUPPORTED_ENCODERS = {"vp8enc", "vp9enc", "vavp9enc"}
PASSTHROUGH = {"videoconvert", "cudaupload", "cudaconvert", "cudadownload", "vapostproc", "hipupload",
               "hipconvert", "queue", "videorate", "capsfilter", "identity", "audioconvert", "audioresample",
               "tee", "fakesink"}


class PipelineError(ValueError):
    pass


@dataclass
class Element:
    name: str
    props: dict = field(default_factory=dict)
    features: str = ""   # caps features, e.g. "memory:CUDAMemory"


@dataclass
class PipelineSpec:
    source: str = "x11"                 # x11 | synthetic
    display: Optional[str] = None
    show_pointer: bool = True
    region: Optional[tuple] = None      # (x0, y0, x1, y1) inclusive, ximagesrc start/end
    width: Optional[int] = None
    height: Optional[int] = None
    framerate: Optional[float] = None
    encoder: Optional[str] = None       # "h264" | "h265" | "av1" | "jpeg"
    encoder_element: Optional[str] = None
    bitrate_kbps: Optional[int] = None
    keyframe_distance: Optional[int] = None
    qp: Optional[int] = None
    mtu: int = 1200
    stun_server: Optional[str] = None
    audio: bool = False
    audio_device: Optional[str] = None
    audio_bitrate: Optional[int] = None
    audio_frame_ms: Optional[float] = None
    elements: list = field(default_factory=list)


def _split_links(text: str) -> list[str]:
    out, cur, quote = [], [], None
    for ch in text:
        if quote:
            cur.append(ch)
            if ch == quote:
                quote = None
        elif ch in "\"'":
            quote = ch
            cur.append(ch)
        elif ch == "!":
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur).strip())
    if any(not s for s in out):
        raise PipelineError("empty element between '!' links")
    return out


def _value(v: str):
    v = v.strip()
    if len(v) >= 2 and v[0] == v[-1] and v[0] in "\"'":
        return v[1:-1]
    low = v.lower()
    if low in ("true", "false"):
        return low == "true"
    if "/" in v and all(p.strip("-").isdigit() for p in v.split("/", 1)):
        n, d = v.split("/", 1)
        return int(n) / max(1, int(d))
    try:
        return int(v)
    except ValueError:
        try:
            return float(v)
        except ValueError:
            return v


def _caps(seg: str) -> Element:
    parts = [p.strip() for p in seg.split(",")]
    feats = parts[0].split("(", 1)[1].rstrip(")") if "(" in parts[0] else ""
    parts[0] = parts[0].split("(", 1)[0]   # caps features: video/x-raw(memory:CUDAMemory|VAMemory)
    props = {}
    for p in parts[1:]:
        if "=" in p:
            k, v = p.split("=", 1)
            v = v.split(")", 1)[-1] if v.startswith("(") else v   # (int)1920 / (fraction)60/1
            props[k.strip()] = _value(v)
    return Element(parts[0], props, feats)


def parse_elements(text: str) -> list[Element]:
    """Tokenises a gst-launch style description into elements and caps."""
    elems = []
    for seg in _split_links(" ".join(text.split())):
        first = seg.split(None, 1)[0]
        if "/" in first.split(",")[0] and "=" not in first.split(",")[0]:
            elems.append(_caps(seg))
            continue
        toks = shlex.split(seg)
        e = Element(toks[0])
        for t in toks[1:]:
            if "=" not in t:
                raise PipelineError(f"bad property {t!r} on {e.name}")
            k, v = t.split("=", 1)
            e.props[k] = _value(v)
        elems.append(e)
    return elems


def parse_pipeline(text: str) -> PipelineSpec:
    spec = PipelineSpec()
    spec.elements = parse_elements(text)
    for e in spec.elements:
        n, p = e.name, e.props
        if n == "ximagesrc":
            spec.source = "x11"
            spec.display = p.get("display-name")
            spec.show_pointer = bool(p.get("show-pointer", True))
            if any(k in p for k in ("startx", "starty", "endx", "endy")):
                spec.region = (int(p.get("startx", 0)), int(p.get("starty", 0)), int(p.get("endx", 0)),
                               int(p.get("endy", 0)))
        elif n in ("videotestsrc", "hipsrc"):
            spec.source = "synthetic"
        elif n.startswith("video/"):
            if n != "video/x-raw":
                raise PipelineError(f"caps {n}: only raw video caps may precede the encoder")
            spec.width = p.get("width", spec.width)
            spec.height = p.get("height", spec.height)
            if "framerate" in p:
                spec.framerate = float(p["framerate"])
        elif n in H264_ENCODERS or n in H265_ENCODERS or n in AV1_ENCODERS:
            spec.encoder = "h265" if n in H265_ENCODERS else ("av1" if n in AV1_ENCODERS else "h264")
            spec.encoder_element = n
            for k in ("bitrate", "target-bitrate"):
                if k in p:
                    spec.bitrate_kbps = int(p[k]) // (1000 if n == "rav1enc" else 1)   # rav1enc: bit/s
            for k in ("key-int-max", "gop-size", "keyframe-period", "idr-period"):
                if k in p and int(p[k]) > 0:
                    spec.keyframe_distance = int(p[k])
            for k in ("quantizer", "qp-const", "qp", "qp-i"):
                if k in p:
                    spec.qp = int(p[k])
        elif n == "jpegenc":
            spec.encoder, spec.encoder_element = "jpeg", n
        elif n in UNSUPPORTED_ENCODERS:
            raise PipelineError(f"{n}: this build encodes H.264 / H.265 / AV1 (HIP) and JPEG; use one of "
                                "those encoder elements")
        elif n in ("rtph264pay", "rtph265pay", "rtpav1pay", "rtpopuspay"):
            if "mtu" in p:
                spec.mtu = int(p["mtu"])
        elif n == "webrtcbin":
            spec.stun_server = p.get("stun-server")
        elif n == "pulsesrc":
            spec.audio = True
            spec.audio_device = p.get("device")
        elif n == "opusenc":
            spec.audio = True
            if "bitrate" in p:
                spec.audio_bitrate = int(p["bitrate"])
            if "frame-size" in p:
                spec.audio_frame_ms = float(p["frame-size"])
        elif n.startswith("audio/"):
            pass
        elif n not in PASSTHROUGH:
            raise PipelineError(f"unknown element {n!r}")
    return spec


def apply_to_args(spec: PipelineSpec, args) -> None:
    """Overrides the legacy app's argparse namespace with what the pipeline sets."""
    if spec.encoder == "jpeg":
        raise PipelineError("jpegenc is for the websocket mode; WebRTC carries H.264")
    if spec.encoder_element:
        args.encoder = spec.encoder_element
    if spec.framerate:
        args.framerate = str(int(round(spec.framerate)))
    if spec.bitrate_kbps:
        args.video_bitrate = str(spec.bitrate_kbps)
    if spec.keyframe_distance:
        args.keyframe_distance = str(spec.keyframe_distance)
    if spec.width and spec.height:
        args.initial_resolution = f"{spec.width}x{spec.height}"
    if spec.audio_bitrate:
        args.audio_bitrate = str(spec.audio_bitrate)
    if hasattr(args, "capture_source"):
        args.capture_source = spec.source
    if hasattr(args, "enable_cursors"):
        args.enable_cursors = "false" if spec.show_pointer else "true"   # server-side cursor vs client cursors


# ---------------------------------------------------------------------------
# Real GStreamer (gst-launch-1.0 + libgsthip)
GST_ENCODER_FOR = {**{n: "hiph264enc" for n in H264_ENCODERS}, **{n: "hiph265enc" for n in H265_ENCODERS},
                   **{n: "hipav1enc" for n in AV1_ENCODERS}}
# the reference's GPU memory elements map to libgsthip's (device frames as memory:HIPMemory):
# cudaupload / cudaconvert / cudadownload (gstwebrtc_app.py:261-284); ximagesrc (not in this
# image's GStreamer) to hipximagesrc with the same properties
GST_RENAME = {"cudaupload": "hipupload", "cudaconvert": "hipconvert", "cudadownload": "hipdownload",
              "ximagesrc": "hipximagesrc"}
GST_CAPS_FEATURES = {"memory:CUDAMemory": "memory:HIPMemory", "memory:VAMemory": "memory:HIPMemory"}
# VA post-processing has no counterpart: the encoders convert BGRx themselves
GST_DROP = {"vapostproc"}
GST_NO_ELEMENT = {"webrtcbin", "rtph264pay", "rtph265pay", "rtpav1pay", "rtpopuspay", "pulsesrc", "opusenc"}
# ximagesrc properties hipximagesrc does not take (xid / xname windows are not captured)
GST_XIMAGESRC_PROPS = {"display-name", "show-pointer", "use-damage", "startx", "starty", "endx", "endy", "remote"}


def _gst_value(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return str(v)


def _gst_encoder_props(name: str, p: dict) -> list[str]:
    out = []
    for k in ("bitrate", "target-bitrate"):
        if k in p:
            out.append(f"bitrate={int(p[k]) // (1000 if name == 'rav1enc' else 1)}")
            break
    for k in ("key-int-max", "gop-size", "keyframe-period", "idr-period", "keyframe-max-dist",
              "intra-period-length", "max-key-frame-interval"):
        if k in p:
            v = int(p[k])
            out.append(f"key-int-max={v if 0 < v < 2 ** 31 - 1 else -1}")
            break
    for k in ("quantizer", "qp-const", "qp"):
        if k in p:
            out.append(f"qp={int(p[k])}")
            break
    mode = str(p.get("rc-mode", p.get("pass", p.get("end-usage", p.get("rate-control", ""))))).lower()
    if "cbr" in mode:
        out.append("rate-control=cbr")
    elif mode in ("cqp", "constqp", "quant", "qp"):
        out.append("rate-control=cqp")
    return out


def to_gst_launch(text: str) -> list[str]:
    """gst-launch-1.0 arguments for a launch string, with this build's GStreamer elements
    in place of the reference's encoders (see the module docstring)."""
    out: list[str] = []
    for e in parse_elements(text):
        n, p = e.name, e.props
        if n in UNSUPPORTED_ENCODERS:
            raise PipelineError(f"{n}: this build encodes H.264 / H.265 / AV1 (HIP) and JPEG")
        if n in GST_NO_ELEMENT:
            raise PipelineError(f"{n}: not in this GStreamer build; WebRTC runs on the own stack (legacy app)")
        if n in GST_DROP:
            continue
        if n.startswith("video/") or n.startswith("audio/"):
            feats = GST_CAPS_FEATURES.get(e.features, e.features)
            if feats == "memory:HIPMemory" and not _hip_devices():
                feats = ""   # CPU-only host: hipupload / hipconvert keep frames in system memory
            head = f"{n}({feats})" if feats else n
            caps = [head] + [f"{k}={_gst_value(v) if k != 'framerate' else _gst_framerate(v)}" for k, v in p.items()]
            seg = [",".join(caps)]
        elif n in GST_ENCODER_FOR:
            seg = [GST_ENCODER_FOR[n], *_gst_encoder_props(n, p)]
        elif n == "ximagesrc":
            seg = ["hipximagesrc", *(f"{k}={_gst_value(v)}" for k, v in p.items() if k in GST_XIMAGESRC_PROPS)]
        else:
            seg = [GST_RENAME.get(n, n), *(f"{k}={_gst_value(v)}" for k, v in p.items())]
        if out:
            out.append("!")
        out.extend(seg)
    return out


def _hip_devices() -> int:
    try:
        from selkies_gstreamer_amd.ops.native import hip_device_count
        return hip_device_count()
    except (OSError, RuntimeError):
        return 0


def _gst_framerate(v) -> str:
    from fractions import Fraction
    f = Fraction(float(v)).limit_denominator(1001)
    return f"{f.numerator}/{f.denominator}"


def gst_available() -> bool:
    try:
        from selkies_gstreamer_amd.ops import build_gst
    except ImportError:
        return False
    return build_gst.available() and build_gst.PLUGIN.exists()


def run_gst(text: str, timeout: float | None = None):
    """Runs a launch string in real GStreamer (gst-launch-1.0 with libgsthip); returns the
    CompletedProcess. Raises PipelineError when GStreamer or the plugin is absent."""
    import subprocess
    if not gst_available():
        raise PipelineError("GStreamer with libgsthip is not available (ops/build_gst.py)")
    from selkies_gstreamer_amd.ops import build_gst
    return subprocess.run([build_gst.gst_bin("gst-launch-1.0"), "-q", *to_gst_launch(text)],
                          env=build_gst.gst_env(), capture_output=True, text=True, timeout=timeout)

