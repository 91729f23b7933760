"""GStreamer launch-string front end of the legacy mode (legacy/pipeline.py):
the reference's own encoder chains map onto the HIP engine."""
import pytest

from selkies_gstreamer_amd.legacy.pipeline import PipelineError, parse_elements, parse_pipeline
from selkies_gstreamer_amd.legacy.webrtc_app import parse_args

X264 = ('ximagesrc display-name=:0 show-pointer=true use-damage=0 remote=true blocksize=16384 ! '
        'video/x-raw,framerate=60/1 ! videoconvert n-threads=4 ! video/x-raw,format=NV12 ! '
        'x264enc threads=4 bframes=0 key-int-max=0 mb-tree=false rc-lookahead=0 sliced-threads=true '
        'byte-stream=true pass=cbr speed-preset=ultrafast tune=zerolatency bitrate=8000 ! '
        'rtph264pay mtu=1200 aggregate-mode=zero-latency config-interval=-1 ! webrtcbin name=app '
        'stun-server=stun://stun.l.google.com:19302')
NVENC = ('ximagesrc show-pointer=false ! cudaupload ! cudaconvert ! '
         'video/x-raw(memory:CUDAMemory),format=NV12 ! nvh264enc bitrate=12000 rc-mode=cbr gop-size=120 '
         'preset=p4 tune=ultra-low-latency ! rtph264pay mtu=1000')


def test_x264_chain():
    s = parse_pipeline(X264)
    assert (s.source, s.display, s.show_pointer) == ("x11", ":0", True)
    assert s.framerate == 60 and s.encoder == "h264" and s.encoder_element == "x264enc"
    assert s.bitrate_kbps == 8000 and s.keyframe_distance is None and s.mtu == 1200
    assert s.stun_server == "stun://stun.l.google.com:19302"


def test_nvenc_chain_and_caps_features():
    s = parse_pipeline(NVENC)
    assert s.encoder_element == "nvh264enc" and s.bitrate_kbps == 12000 and s.keyframe_distance == 120
    assert s.mtu == 1000 and not s.show_pointer


def test_audio_branch_and_region():
    s = parse_pipeline('ximagesrc startx=0 starty=0 endx=1279 endy=719 ! video/x-raw,width=1280,height=720,'
                       'framerate=(fraction)30/1 ! hiph264enc qp-const=22 ! rtph264pay')
    assert s.region == (0, 0, 1279, 719) and (s.width, s.height, s.framerate, s.qp) == (1280, 720, 30.0, 22)
    a = parse_pipeline('pulsesrc device=output.monitor ! audioconvert ! opusenc bitrate=128000 frame-size=10 ! '
                       'rtpopuspay mtu=1200')
    assert a.audio and a.audio_device == "output.monitor" and a.audio_bitrate == 128000 and a.audio_frame_ms == 10


@pytest.mark.parametrize("enc", ["vp8enc", "vp9enc", "vavp9enc"])
def test_unsupported_codecs_are_explicit(enc):
    with pytest.raises(PipelineError, match="H.264"):
        parse_pipeline(f"ximagesrc ! videoconvert ! {enc} ! fakesink")


@pytest.mark.parametrize("enc,prop,val,kbps", [("svtav1enc", "target-bitrate", 6000, 6000),
                                               ("rav1enc", "bitrate", 6000000, 6000),
                                               ("nvav1enc", "bitrate", 6000, 6000)])
def test_av1_encoders_map_to_hip_av1(enc, prop, val, kbps):
    s = parse_pipeline(f"ximagesrc ! videoconvert ! {enc} {prop}={val} ! rtpav1pay mtu=1200")
    assert (s.encoder, s.encoder_element, s.bitrate_kbps, s.mtu) == ("av1", enc, kbps, 1200)


def test_syntax_errors():
    with pytest.raises(PipelineError):
        parse_pipeline("ximagesrc ! ! x264enc")
    with pytest.raises(PipelineError):
        parse_pipeline("ximagesrc ! frobnicate ! x264enc")
    assert [e.name for e in parse_elements('a b="x ! y" ! c')] == ["a", "c"]


def test_legacy_args_take_pipeline_settings():
    args = parse_args(["--json_config", "/nonexistent.json", "--video_pipeline",
                       'videotestsrc ! video/x-raw,width=1280,height=720,framerate=30/1 ! '
                       'vah264enc bitrate=4000 key-int-max=60 ! rtph264pay'], env={})
    assert (args.encoder, args.framerate, args.video_bitrate, args.keyframe_distance) == ("vah264enc", "30", "4000", "60")
    assert args.initial_resolution == "1280x720" and args.capture_source == "synthetic"
