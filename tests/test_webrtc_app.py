"""Legacy WebRTC mode end to end on CPU: signalling server + streaming peer
(synthetic capture, CPU H.264 in full-frame mode) <-> a viewer peer built from
our own PeerConnection acting as the browser. Checks the signalling call
flow (HELLO / SESSION / SDP relay), DTLS-SRTP media (decodable IDR), the
"input" data channel in both directions and runtime bitrate / fps control."""
import asyncio
import json

import pytest

from selkies_gstreamer_amd.legacy import webrtc_app
from selkies_gstreamer_amd.legacy.signalling_client import SignallingClient
from selkies_gstreamer_amd.models.h264.decoder import H264Decoder
from selkies_gstreamer_amd.webrtc.peer import PeerConnection


class _RecordingInput:
    def __init__(self):
        self.msgs = []

    async def on_message(self, msg):
        self.msgs.append(msg)

    async def close(self):
        pass


@pytest.mark.parametrize("backend,encoder", [("cpu", "x264enc"), ("cpu", "svtav1enc"),
                                             pytest.param("hip", "x264enc", marks=pytest.mark.gpu),
                                             pytest.param("hip", "svtav1enc", marks=pytest.mark.gpu)])
def test_legacy_webrtc_session(tmp_path, backend, encoder):
    """backend=hip runs the same session on the MI355X encoder (native HIP path, 640x368);
    encoder=svtav1enc carries AV1 over RTP (rtpav1pay payload format) and the viewer's
    temporal units are decoded by dav1d."""
    W, H = (256, 128) if backend == "cpu" else (640, 368)
    args = webrtc_app.parse_args(
        ["--port", "0", "--enable_basic_auth", "false", "--use_cpu", str(backend == "cpu").lower(),
         "--capture_source", "synthetic", "--json_config", str(tmp_path / "cfg.json"),
         "--rtc_config_json", str(tmp_path / "none.json"), "--framerate", "20", "--encoder", encoder,
         "--initial_resolution", f"{W}x{H}", "--turn_shared_secret", ""], env={})
    rec = _RecordingInput()

    async def factory(session):
        return rec

    async def main():
        stop = asyncio.Event()
        srv = asyncio.ensure_future(webrtc_app.serve(args, factory, addresses=["127.0.0.1"], stop=stop))
        for _ in range(100):
            if args.port != "0":
                break
            await asyncio.sleep(0.05)
        viewer = PeerConnection(addresses=["127.0.0.1"])
        frames, msgs, chans = [], [], []
        viewer.on_video_frame = lambda au, ts: frames.append(au)

        def on_channel(ch):
            chans.append(ch)
            ch.on_message = msgs.append
        viewer.on_datachannel = on_channel
        sig = SignallingClient(f"ws://127.0.0.1:{args.port}/ws", 1)
        answered = asyncio.Event()
        offers = {}

        async def on_offer(kind, text):
            offers["video"] = text
            await viewer.set_remote_description(text, kind)
            await sig.send_sdp("answer", await viewer.create_answer())
            answered.set()
            await viewer.connect(15)
        sig.on_sdp = lambda kind, text: asyncio.ensure_future(on_offer(kind, text))
        await sig.connect()
        reader = asyncio.ensure_future(sig.start())
        await asyncio.wait_for(answered.wait(), 20)
        def is_key(f):   # AV1 temporal unit carrying a sequence header (key frame)
            return len(f) > 2 and (f[2] >> 3) & 15 == 1
        pli = False
        for _ in range(600):   # up to 30 s: a HIP AV1 session's first frames include device warm-up
            if len(frames) >= 5 and chans and msgs and (encoder != "svtav1enc" or any(map(is_key, frames))):
                break
            if encoder == "svtav1enc" and len(frames) >= 3 and not pli and not any(map(is_key, frames)):
                # the first key frame can go out before this viewer's SRTP is up: ask for one (PLI)
                viewer.request_keyframe(next(iter(viewer._depack)))
                pli = True
            await asyncio.sleep(0.05)
        assert len(frames) >= 5, "no video over SRTP"
        if encoder == "svtav1enc":
            from selkies_gstreamer_amd.models.av1 import dav1d
            assert frames[0][:2] == b"\x12\x00"          # temporal unit rebuilt by AV1Depacketizer
            keys = [i for i, f in enumerate(frames) if is_key(f)]   # sequence header
            assert keys, "no key frame received"
            if dav1d.available():
                d = dav1d.Decoder()
                pics = [d.decode(f) for f in frames[keys[0]:]]
                assert pics[0] is not None and pics[0][0].shape == (H, W)
        else:
            dec = H264Decoder()
            out = []
            for au in frames[:3]:
                out += dec.decode(au)
            assert out and out[0][0].shape == (H, W) and dec.stats["idr"] >= 1
        sysmsgs = [json.loads(m) for m in msgs]
        assert {"type": "system", "data": {"action": "framerate,20"}} in sysmsgs
        ch = chans[0]
        assert ch.label == "input"
        ch.send("kd,65")
        ch.send("vb,2500")
        ch.send("_arg_fps,30")
        for _ in range(100):
            if rec.msgs and any("Video bitrate set to: 2500" in m for m in msgs):
                break
            await asyncio.sleep(0.05)
        assert rec.msgs == ["kd,65"]
        assert any("Video bitrate set to: 2500" in m for m in msgs)
        saved = json.loads((tmp_path / "cfg.json").read_text())
        assert saved["video_bitrate"] == "2500" and saved["framerate"] == "30"
        # the second peer (uid 3) gets its own audio-only call from uid 2 (reference two-peer
        # client, app.js:375-378); the video call carries no audio section
        assert "m=video" in offers["video"] and "m=audio" not in offers["video"]
        aviewer = PeerConnection(addresses=["127.0.0.1"])
        asig = SignallingClient(f"ws://127.0.0.1:{args.port}/ws", 3)
        aconnected = asyncio.Event()

        async def on_audio_offer(kind, text):
            offers["audio"] = text
            await aviewer.set_remote_description(text, kind)
            await asig.send_sdp("answer", await aviewer.create_answer())
            await aviewer.connect(15)
            aconnected.set()
        asig.on_sdp = lambda kind, text: asyncio.ensure_future(on_audio_offer(kind, text))
        await asig.connect()
        areader = asyncio.ensure_future(asig.start())
        await asyncio.wait_for(aconnected.wait(), 20)
        assert "m=audio" in offers["audio"] and "m=video" not in offers["audio"]
        assert "m=application" not in offers["audio"]
        await aviewer.close()
        areader.cancel()
        await asig.stop()
        await viewer.close()
        reader.cancel()
        await sig.stop()
        stop.set()
        await asyncio.wait_for(srv, 15)

    asyncio.run(asyncio.wait_for(main(), 120))
