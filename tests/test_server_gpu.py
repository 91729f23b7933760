"""GPU twin of test_server_e2e.py: a live data-websocket session whose capture
session runs the HIP encoder (no --use-cpu), decoded stripe by stripe with the
independent test decoder, plus the frame-trace path (FRAME_TS grab timestamps)
that tools/bench_e2e.py measures capture -> client latency with."""
import asyncio
import json
import time

import aiohttp
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import hip_device_count
from selkies_gstreamer_amd.server.data_server import DataStreamingServer
from selkies_gstreamer_amd.server.settings import Settings
from tests.h264_util import StripeDecoder, bgrx_to_y709, psnr

pytestmark = pytest.mark.gpu


def _native():
    import ctypes
    from selkies_gstreamer_amd.ops import native
    L = native.lib()
    L.sk_synthetic_render.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p]
    L.sk_synthetic_render.restype = ctypes.c_int
    return L


@pytest.fixture(autouse=True)
def _need_gpu():
    if hip_device_count() < 1:
        pytest.skip("no HIP device")


async def _recv_until(ws, pred, timeout=30.0):
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


@pytest.mark.parametrize("W,H,encoder", [(1920, 1080, "x264enc-striped"), (1280, 720, "x264enc")])
def test_hip_session_decodes(tmp_path, W, H, encoder):
    async def main():
        s = Settings(["--port", "0", "--audio-enabled", "false"], env={})
        srv = DataStreamingServer(s, upload_dir=str(tmp_path / "up"), capture_source="motion", frame_trace=True)
        port = await srv.start("127.0.0.1", 0)
        try:
            async with aiohttp.ClientSession() as sess:
                async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket", max_msg_size=0) as ws:
                    await _recv_until(ws, lambda m: isinstance(m, str) and "server_settings" in m)
                    await ws.send_str("SETTINGS," + json.dumps({"initialClientWidth": W, "initialClientHeight": H,
                                                                 "framerate": 60, "encoder": encoder}))
                    dec = StripeDecoder(W, H)
                    grabs, lat, frames, pkts = {}, [], set(), []
                    keyed = False
                    end = time.monotonic() + 40
                    while len(frames) < 30 and time.monotonic() < end:
                        msg = await asyncio.wait_for(ws.receive(), 30)
                        now = time.monotonic_ns()
                        d = msg.data
                        if isinstance(d, str):
                            if d.startswith("FRAME_TS "):
                                _, fid, g = d.split()
                                grabs[int(fid)] = int(g)
                            continue
                        if not isinstance(d, bytes) or d[0] != 0x04:
                            continue
                        keyed = keyed or d[1] == 1
                        if not keyed:
                            continue  # joined mid-GOP: wait for the first IDR
                        fid = int.from_bytes(d[2:4], "big")
                        if len(frames) < 3 or (fid in frames and len(frames) == 3):
                            pkts.append(d)  # first 3 frames; decoded after the run (the Python decoder is slow)
                        if fid not in frames:
                            frames.add(fid)
                            if fid in grabs:
                                lat.append((now - grabs.pop(fid)) / 1e6)
                            await ws.send_str(f"CLIENT_FRAME_ACK {fid}")
                    assert len(frames) >= 30
                    for d in pkts:
                        dec.feed(d)
                    assert dec.Y.std() > 5.0
                    # the picture after the last fed frame against the exact frame the session
                    # captured (the native synthetic source, rendered again for that frame id)
                    fid = int.from_bytes(pkts[-1][2:4], "big")
                    ref = np.empty((H, W, 4), np.uint8)
                    assert _native().sk_synthetic_render(W, H, 0, fid, ref.ctypes.data) == 0
                    q = psnr(dec.Y, bgrx_to_y709(ref))
                    assert q > 30.0, f"decoded frame {fid}: {q:.2f} dB against its source"
                    assert lat, "no FRAME_TS traces"
                    # capture -> receive must be a few frame intervals at most on one host
                    assert float(np.median(lat)) < 100.0, lat
                    assert srv.displays["primary"].flow.acknowledged >= 0
        finally:
            await srv.stop()
    asyncio.run(asyncio.wait_for(main(), 120))


def test_session_host_two_hip_sessions():
    """parallel/multi.py: two servers in one process share the HIP context; both
    stream decodable H.264 at their own sizes at the same time."""
    import socket
    from selkies_gstreamer_amd.parallel.multi import host

    def free_port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    async def client(port, W, H):
        async with aiohttp.ClientSession() as sess:
            async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket", max_msg_size=0) as ws:
                await _recv_until(ws, lambda m: isinstance(m, str) and "server_settings" in m)
                await ws.send_str("SETTINGS," + json.dumps({"initialClientWidth": W, "initialClientHeight": H,
                                                             "framerate": 60, "encoder": "x264enc"}))
                dec = StripeDecoder(W, H)
                frames = 0
                while frames < 2:
                    d, _ = await _recv_until(ws, lambda m: isinstance(m, bytes) and m[0] == 0x04 and
                                             (frames > 0 or m[1] == 1))
                    dec.feed(d)
                    frames += 1
                return dec.Y.std(), int.from_bytes(d[6:8], "big")

    async def main():
        ports = [free_port(), free_port()]
        up, stop = [], asyncio.Event()
        task = asyncio.create_task(host(ports, ["--host", "127.0.0.1", "--capture-source", "motion",
                                                "--audio-enabled", "false", "--gamepad-enabled", "false"],
                                        stop=stop, ready=lambda srv, port: up.append(port)))
        try:
            for _ in range(600):
                if len(up) == 2:
                    break
                await asyncio.sleep(0.05)
            assert sorted(up) == sorted(ports)
            (s0, w0), (s1, w1) = await asyncio.wait_for(asyncio.gather(client(ports[0], 640, 368),
                                                                        client(ports[1], 1280, 720)), 60)
            assert (w0, w1) == (640, 1280) and s0 > 5.0 and s1 > 5.0
        finally:
            stop.set()
            await asyncio.wait_for(task, 30)
    asyncio.run(main())


def test_hip_session_hevc_decodes(tmp_path):
    """HEVC (x265enc) over the data websocket from the HIP encoder: the first frames from
    the key frame decode with the independent HEVC decoder and match their source."""
    from selkies_gstreamer_amd.models.hevc.decoder import HevcDecoder
    W, H = 640, 368

    async def main():
        s = Settings(["--port", "0", "--audio-enabled", "false"], env={})
        srv = DataStreamingServer(s, upload_dir=str(tmp_path / "up"), capture_source="motion")
        port = await srv.start("127.0.0.1", 0)
        pkts = []
        try:
            async with aiohttp.ClientSession() as sess:
                async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket", max_msg_size=0) as ws:
                    await _recv_until(ws, lambda m: isinstance(m, str) and "server_settings" in m)
                    await ws.send_str("SETTINGS," + json.dumps({"initialClientWidth": W, "initialClientHeight": H,
                                                                 "framerate": 60, "encoder": "x265enc"}))
                    end = time.monotonic() + 40
                    while len(pkts) < 3 and time.monotonic() < end:
                        d = (await asyncio.wait_for(ws.receive(), 30)).data
                        if not isinstance(d, bytes) or d[0] != 0x04 or (not pkts and d[1] != 1):
                            continue
                        pkts.append(d)
                        await ws.send_str(f"CLIENT_FRAME_ACK {int.from_bytes(d[2:4], 'big')}")
        finally:
            await srv.stop()
        return pkts

    pkts = asyncio.run(asyncio.wait_for(main(), 120))
    assert len(pkts) == 3
    dec = HevcDecoder()
    pics = [p for d in pkts for p in dec.decode(d[10:])]
    assert len(pics) == 3
    fid = int.from_bytes(pkts[-1][2:4], "big")
    ref = np.empty((H, W, 4), np.uint8)
    assert _native().sk_synthetic_render(W, H, 0, fid, ref.ctypes.data) == 0
    q = psnr(pics[-1][0].astype(np.float64), bgrx_to_y709(ref))
    assert q > 30.0, f"decoded frame {fid}: {q:.2f} dB against its source"
