"""End-to-end data-websocket sessions against a live server (aiohttp client).

The server runs with the synthetic capture source and the CPU reference
encoders (``--use-cpu true``) so the full path — SETTINGS -> display layout ->
native capture session -> stripe packets -> websocket -> decode — runs on CPU.
The GPU twin of this test lives in test_server_gpu.py.
"""
import asyncio
import json
import os
import time

import aiohttp
import numpy as np
import pytest

from selkies_gstreamer_amd.server.data_server import DataStreamingServer
from selkies_gstreamer_amd.server.input import InputHandler, RecordingInjector
from selkies_gstreamer_amd.server.settings import Settings
from tests.h264_util import StripeDecoder


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 60))


async def _server(tmp_path, argv=(), with_input=False):
    s = Settings(["--port", "0", "--use-cpu", "true", "--audio-enabled", "false", *argv], env={})
    rec = RecordingInjector()

    async def factory(server):
        return InputHandler(rec)
    srv = DataStreamingServer(s, upload_dir=str(tmp_path / "up"), capture_source="synthetic",
                              input_factory=factory if with_input else None)
    port = await srv.start("127.0.0.1", 0)
    return srv, port, rec


async def _recv_until(ws, pred, timeout=10.0):
    """Reads messages until pred(msg) is true; returns (match, all_messages)."""
    seen = []
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while True:
        msg = await asyncio.wait_for(ws.receive(), max(0.01, end - loop.time()))
        if msg.type in (aiohttp.WSMsgType.CLOSE, aiohttp.WSMsgType.CLOSED, aiohttp.WSMsgType.ERROR):
            raise ConnectionError(f"closed: {msg}")
        seen.append(msg.data)
        if pred(msg.data):
            return msg.data, seen


def _settings(w=256, h=128, **kw):
    d = {"initialClientWidth": w, "initialClientHeight": h, "framerate": 30, "encoder": "x264enc-striped"}
    d.update(kw)
    return "SETTINGS," + json.dumps(d)


def test_session_h264_striped(tmp_path):
    async def main():
        srv, port, _ = await _server(tmp_path)
        async with aiohttp.ClientSession() as sess:
            async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket") as ws:
                first = await ws.receive()
                assert first.data == "MODE websockets"
                ss, _ = await _recv_until(ws, lambda m: isinstance(m, str) and "server_settings" in m)
                assert json.loads(ss)["settings"]["encoder"]["value"] == "x264enc"
                await ws.send_str(_settings())
                res, seen = await _recv_until(ws, lambda m: isinstance(m, str) and "stream_resolution" in m)
                assert json.loads(res) == {"type": "stream_resolution", "width": 256, "height": 128}
                dec = StripeDecoder(256, 128)
                pending = [m for m in seen if isinstance(m, bytes)]
                n = 0
                while n < 8:
                    if pending:
                        data = pending.pop(0)
                    else:
                        data = (await asyncio.wait_for(ws.receive(), 10)).data
                    if isinstance(data, bytes):
                        assert data[0] == 0x04
                        dec.feed(data)
                        fid = int.from_bytes(data[2:4], "big")
                        await ws.send_str(f"CLIENT_FRAME_ACK {fid}")
                        n += 1
                assert srv.displays["primary"].flow.acknowledged >= 0
                assert dec.Y.std() > 1.0  # decoded real content
                # resize -> new resolution broadcast
                await ws.send_str("r,320x160,primary")
                res, _ = await _recv_until(ws, lambda m: isinstance(m, str) and "stream_resolution" in m)
                assert json.loads(res)["width"] == 320
                # stop / start video
                await ws.send_str("STOP_VIDEO")
                await _recv_until(ws, lambda m: m == "VIDEO_STOPPED")
                assert "primary" not in srv.captures
                await ws.send_str("START_VIDEO")
                await _recv_until(ws, lambda m: m == "VIDEO_STARTED")
                assert "primary" in srv.captures
        await asyncio.sleep(0.2)
        assert not srv.captures and not srv.displays
        await srv.stop()
    run(main())


def test_keyframe_request_resyncs_a_viewer(tmp_path):
    """REQUEST_KEYFRAME (sent by web/lib/video.js when its decoder dropped a delta) makes
    the display's next frames start with a 0x04 key frame within a few frames: the frames
    already encoded or queued on the socket when the request lands (up to two under a
    loaded CPU) arrive first."""
    async def main():
        srv, port, _ = await _server(tmp_path)
        async with aiohttp.ClientSession() as sess:
            async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket") as ws:
                await ws.send_str(_settings(encoder="x264enc"))
                frames = []
                while len(frames) < 6:
                    data = (await asyncio.wait_for(ws.receive(), 10)).data
                    if isinstance(data, bytes) and data[0] == 0x04:
                        frames.append(data[1])
                assert frames[0] == 1 and not any(frames[1:])   # one IDR, then P frames
                await ws.send_str("REQUEST_KEYFRAME")
                await ws.send_str("REQUEST_KEYFRAME")             # a second viewer / repeat: one IDR
                after = []
                while len(after) < 10:
                    data = (await asyncio.wait_for(ws.receive(), 10)).data
                    if isinstance(data, bytes) and data[0] == 0x04:
                        after.append(data[1])
                assert 1 in after[:4], after
                assert sum(after) == 1, after
        await srv.stop()
    run(main())


def test_session_jpeg_and_fullframe(tmp_path):
    async def main():
        srv, port, _ = await _server(tmp_path)
        async with aiohttp.ClientSession() as sess:
            async with sess.ws_connect(f"http://127.0.0.1:{port}/") as ws:
                await ws.send_str(_settings(192, 128, encoder="jpeg", jpeg_quality=60))
                data, _ = await _recv_until(ws, lambda m: isinstance(m, bytes))
                assert data[:2] == b"\x03\x00" and data[6:8] == b"\xff\xd8"
                # switch encoder to full-frame H.264 (video params change -> capture restart)
                await ws.send_str(_settings(192, 128, encoder="x264enc"))
                data, _ = await _recv_until(ws, lambda m: isinstance(m, bytes) and m[0] == 0x04)
                assert int.from_bytes(data[4:6], "big") == 0  # full frame: y = 0
        await srv.stop()
    run(main())


def test_takeover_kill_and_debounce(tmp_path):
    async def main():
        srv, port, _ = await _server(tmp_path)
        async with aiohttp.ClientSession() as sess:
            ws1 = await sess.ws_connect(f"http://127.0.0.1:{port}/")
            await ws1.send_str(_settings())
            await _recv_until(ws1, lambda m: isinstance(m, str) and "stream_resolution" in m)
            # immediate reconnect from the same IP -> rate limited
            ws_fast = await sess.ws_connect(f"http://127.0.0.1:{port}/")
            m = await ws_fast.receive()
            assert m.type == aiohttp.WSMsgType.CLOSE and ws_fast.close_code == 4029
            await asyncio.sleep(0.6)
            ws2 = await sess.ws_connect(f"http://127.0.0.1:{port}/")
            await ws2.send_str(_settings())
            kill, _ = await _recv_until(ws1, lambda m: isinstance(m, str) and m.startswith("KILL"))
            assert "primary" in kill
            await _recv_until(ws2, lambda m: isinstance(m, bytes))
            await ws2.close()
            await ws1.close()
        await srv.stop()
    run(main())


def test_second_screen_layout(tmp_path):
    async def main():
        srv, port, _ = await _server(tmp_path)
        async with aiohttp.ClientSession() as sess:
            p = await sess.ws_connect(f"http://127.0.0.1:{port}/")
            await p.send_str(_settings(256, 128))
            await _recv_until(p, lambda m: isinstance(m, bytes))
            await asyncio.sleep(0.6)
            d2 = await sess.ws_connect(f"http://127.0.0.1:{port}/")
            await d2.send_str(_settings(128, 64, displayId="display2", displayPosition="down"))
            cfg, _ = await _recv_until(p, lambda m: isinstance(m, str) and m.startswith("DISPLAY_CONFIG_UPDATE")
                                       and "display2" in m)
            assert json.loads(cfg.split(",", 1)[1])["displays"] == ["primary", "display2"]
            assert srv.layouts["display2"] == {"x": 0, "y": 128, "w": 128, "h": 64}
            # until its SETTINGS lands, a new connection is a view-only (#shared) client of
            # the primary display and may get primary stripes (reference semantics, selkies.py
            # broadcasts to every client not registered as a secondary display); after that
            # only display2's own 128-wide stream arrives
            data, _ = await _recv_until(d2, lambda m: isinstance(m, bytes) and m[0] == 0x04
                                        and int.from_bytes(m[6:8], "big") == 128)
            for _ in range(3):
                data, _ = await _recv_until(d2, lambda m: isinstance(m, bytes) and m[0] == 0x04)
                assert int.from_bytes(data[6:8], "big") == 128  # display2's own stream width
            await d2.close()
            await p.close()
        await srv.stop()
    run(main())


def test_second_screen_refused_when_disabled(tmp_path):
    async def main():
        srv, port, _ = await _server(tmp_path, ["--second-screen", "false"])
        async with aiohttp.ClientSession() as sess:
            ws = await sess.ws_connect(f"http://127.0.0.1:{port}/")
            await ws.send_str(_settings(displayId="display2"))
            kill, _ = await _recv_until(ws, lambda m: isinstance(m, str) and m.startswith("KILL"))
            assert "disabled" in kill
            await ws.close()
        await srv.stop()
    run(main())


def test_frame_trace_timestamps(tmp_path):
    """SELKIES_FRAME_TRACE: every frame's stripes are preceded by FRAME_TS <fid>
    <grab_ns>, a CLOCK_MONOTONIC grab time (tools/bench_e2e.py latency source)."""
    async def main():
        s = Settings(["--port", "0", "--use-cpu", "true", "--audio-enabled", "false"], env={})
        srv = DataStreamingServer(s, upload_dir=str(tmp_path / "up"), capture_source="synthetic", frame_trace=True)
        port = await srv.start("127.0.0.1", 0)
        async with aiohttp.ClientSession() as sess:
            async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket") as ws:
                await ws.send_str(_settings())
                ts = {}
                while len(ts) < 3:
                    m, _ = await _recv_until(ws, lambda m: isinstance(m, str) and m.startswith("FRAME_TS"))
                    _, fid, g = m.split()
                    ts[int(fid)] = int(g)
                    data, _ = await _recv_until(ws, lambda m: isinstance(m, bytes))
                    now = time.monotonic_ns()
                    assert int.from_bytes(data[2:4], "big") == int(fid)
                    assert 0 < now - int(g) < 5_000_000_000
        await srv.stop()
    run(main())


def test_upload_and_commands(tmp_path):
    async def main():
        srv, port, rec = await _server(tmp_path, ["--command-enabled", "false"], with_input=True)
        async with aiohttp.ClientSession() as sess:
            ws = await sess.ws_connect(f"http://127.0.0.1:{port}/")
            await ws.send_str("FILE_UPLOAD_START:docs/a.txt:6")
            await ws.send_bytes(b"\x01abc")
            await ws.send_bytes(b"\x01def")
            await ws.send_str("FILE_UPLOAD_END:docs/a.txt")
            await ws.send_str("FILE_UPLOAD_START:../escape.txt:1")
            await ws.send_bytes(b"\x01x")
            await ws.send_str("FILE_UPLOAD_END:../escape.txt")
            await ws.send_str("FILE_UPLOAD_START:b.bin:10")
            await ws.send_bytes(b"\x01partial")
            await ws.send_str("FILE_UPLOAD_ERROR:b.bin:cancelled")
            await ws.send_str("cmd,touch " + str(tmp_path / "should_not_exist"))
            await ws.send_str("kd,97")
            await ws.send_str("ku,97")
            await asyncio.sleep(0.3)
            await ws.close()
        assert (tmp_path / "up" / "docs" / "a.txt").read_bytes() == b"abcdef"
        assert not (tmp_path / "escape.txt").exists() and not (tmp_path / "up" / "b.bin").exists()
        assert not (tmp_path / "should_not_exist").exists()
        assert rec.events == [("key", 97, True), ("key", 97, False)]
        await srv.stop()
    run(main())


def test_static_and_health(tmp_path):
    async def main():
        web = tmp_path / "web"
        web.mkdir()
        (web / "index.html").write_text("<html>ok</html>")
        s = Settings(["--port", "0"], env={})
        srv = DataStreamingServer(s, capture_source="synthetic", web_root=str(web))
        port = await srv.start("127.0.0.1", 0)
        async with aiohttp.ClientSession() as sess:
            async with sess.get(f"http://127.0.0.1:{port}/") as r:
                assert r.status == 200 and "ok" in await r.text()
            async with sess.get(f"http://127.0.0.1:{port}/health") as r:
                assert r.status == 200
            async with sess.get(f"http://127.0.0.1:{port}/../../etc/passwd") as r:
                assert r.status == 404
        await srv.stop()
    run(main())


def test_files_listing_and_download(tmp_path):
    """The dashboard files panel's ./files/ area: listing (dirs first, escaped names),
    downloads as attachments, dot files hidden, nothing outside the directory."""
    async def main():
        d = tmp_path / "files"
        (d / "sub").mkdir(parents=True)
        (d / "a <b>.txt").write_text("hello")
        (d / "sub" / "x.bin").write_bytes(b"\0\1\2")
        (d / ".secret").write_text("no")
        (tmp_path / "outside.txt").write_text("no")
        s = Settings(["--port", "0"], env={})
        srv = DataStreamingServer(s, capture_source="synthetic", download_dir=str(d))
        port = await srv.start("127.0.0.1", 0)
        base = f"http://127.0.0.1:{port}"
        async with aiohttp.ClientSession() as sess:
            async with sess.get(f"{base}/files/") as r:
                body = await r.text()
                assert r.status == 200 and "text/html" in r.headers["Content-Type"]
                assert body.index("sub/") < body.index("a &lt;b&gt;.txt")
                assert "a%20%3Cb%3E.txt" in body and ".secret" not in body
            async with sess.get(f"{base}/files/a%20%3Cb%3E.txt") as r:
                assert r.status == 200 and await r.text() == "hello"
                assert "attachment" in r.headers["Content-Disposition"]
            async with sess.get(f"{base}/files/sub", allow_redirects=False) as r:
                assert r.status == 302 and r.headers["Location"].endswith("/files/sub/")
            async with sess.get(f"{base}/files/sub/x.bin") as r:
                assert await r.read() == b"\0\1\2"
            for bad in ("/files/.secret", "/files/../outside.txt", "/files/%2e%2e/outside.txt"):
                async with sess.get(base + bad) as r:
                    assert r.status == 404, bad
        await srv.stop()
        srv3 = DataStreamingServer(s, capture_source="synthetic", download_dir=str(d), basic_auth=("u", "pw"))
        port = await srv3.start("127.0.0.1", 0)
        async with aiohttp.ClientSession() as sess:
            async with sess.get(f"http://127.0.0.1:{port}/files/") as r:
                assert r.status == 401 and "Basic" in r.headers["WWW-Authenticate"]
            async with sess.get(f"http://127.0.0.1:{port}/files/", auth=aiohttp.BasicAuth("u", "bad")) as r:
                assert r.status == 401
            async with sess.get(f"http://127.0.0.1:{port}/files/a%20%3Cb%3E.txt", auth=aiohttp.BasicAuth("u", "pw")) as r:
                assert r.status == 200 and await r.text() == "hello"
        await srv3.stop()
        srv2 = DataStreamingServer(s, capture_source="synthetic")   # downloads disabled
        port = await srv2.start("127.0.0.1", 0)
        async with aiohttp.ClientSession() as sess:
            async with sess.get(f"http://127.0.0.1:{port}/files/") as r:
                assert r.status == 404
        await srv2.stop()
    run(main())


def test_basic_auth_guards_every_route(tmp_path):
    """SELKIES_ENABLE_BASIC_AUTH protects the whole server like the reference's nginx
    block (selkies-gstreamer-entrypoint.sh:89): the websocket upgrade, the web root and
    /metrics answer 401 without credentials; /health stays open; an empty password is
    refused at startup (legacy/signalling_web.py:157-159)."""
    from selkies_gstreamer_amd.server.app import basic_auth_from_env
    from selkies_gstreamer_amd.server.metrics import Metrics

    async def main():
        web = tmp_path / "web"
        web.mkdir()
        (web / "index.html").write_text("<html>ok</html>")
        s = Settings(["--port", "0"], env={})
        srv = DataStreamingServer(s, capture_source="synthetic", web_root=str(web), metrics=Metrics(),
                                  basic_auth=("u", "pw"))
        port = await srv.start("127.0.0.1", 0)
        base = f"http://127.0.0.1:{port}"
        good = aiohttp.BasicAuth("u", "pw")
        async with aiohttp.ClientSession() as sess:
            for path in ("/", "/index.html", "/metrics"):
                async with sess.get(base + path) as r:
                    assert r.status == 401, path
                async with sess.get(base + path, auth=aiohttp.BasicAuth("u", "nope")) as r:
                    assert r.status == 401, path
            async with sess.get(base + "/", auth=good) as r:
                assert r.status == 200 and "ok" in await r.text()
            async with sess.get(base + "/health") as r:
                assert r.status == 200
            with pytest.raises(aiohttp.WSServerHandshakeError) as ei:
                async with sess.ws_connect(base + "/"):
                    pass
            assert ei.value.status == 401
            async with sess.ws_connect(base + "/", auth=good) as ws:
                msg = await ws.receive(timeout=10)
                assert msg.type in (aiohttp.WSMsgType.TEXT, aiohttp.WSMsgType.BINARY)
        await srv.stop()
    run(main())
    with pytest.raises(ValueError):
        DataStreamingServer(Settings(["--port", "0"], env={}), capture_source="synthetic", basic_auth=("u", ""))
    assert basic_auth_from_env({"SELKIES_ENABLE_BASIC_AUTH": "true", "SELKIES_BASIC_AUTH_USER": "a",
                                "SELKIES_BASIC_AUTH_PASSWORD": "b"}) == ("a", "b")


@pytest.mark.parametrize("encoder", ["x265enc", "svtav1enc"])
def test_session_hevc_and_av1(tmp_path, encoder):
    """The MI355X encoder extensions over the data websocket: full-frame HEVC (Annex B,
    in-band parameter sets) and AV1 (OBU temporal units) in the same 0x04 framing; the
    stream decodes with the independent HEVC decoder / dav1d from its first key frame."""
    async def main():
        srv, port, _ = await _server(tmp_path)
        W, H = 192, 128
        frames = []
        async with aiohttp.ClientSession() as sess:
            async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket") as ws:
                ss, _ = await _recv_until(ws, lambda m: isinstance(m, str) and "server_settings" in m)
                assert encoder in json.loads(ss)["settings"]["encoder"]["allowed"]
                await ws.send_str(_settings(W, H, encoder=encoder))
                while len(frames) < 4:
                    data, _ = await _recv_until(ws, lambda m: isinstance(m, bytes) and m[0] == 0x04)
                    assert int.from_bytes(data[4:6], "big") == 0            # full frame: y = 0
                    if frames or data[1] == 1:                             # from the first key frame
                        frames.append(data)
                    await ws.send_str(f"CLIENT_FRAME_ACK {int.from_bytes(data[2:4], 'big')}")
        await srv.stop()
        return frames

    frames = run(main())
    if encoder == "x265enc":
        from selkies_gstreamer_amd.models.hevc.decoder import HevcDecoder
        dec = HevcDecoder()
        pics = [p for f in frames for p in dec.decode(f[10:])]
        assert len(pics) == 4 and pics[0][0].shape == (128, 192) and pics[-1][0].std() > 1.0
    else:
        from selkies_gstreamer_amd.models.av1 import dav1d
        if not dav1d.available():
            pytest.skip("dav1d (libavif) not in this image")
        d = dav1d.Decoder()
        pics = [d.decode(f[10:]) for f in frames]
        assert pics[0] is not None and pics[0][0].shape == (128, 192)
