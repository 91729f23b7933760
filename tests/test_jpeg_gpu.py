"""HIP (gfx950) JPEG stripe encoder: byte-exact against the CPU reference and
decodable by libjpeg (PIL); capture session + websocket server on the GPU."""
import asyncio
import io
import json
import threading
import time

import numpy as np
import pytest
from PIL import Image

from selkies_gstreamer_amd.ops.native import JpegEncoder, lib
from tests.h264_util import StripeDecoder, synthetic_frames

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,sh,kind", [(192, 128, 64, "desktop"), (250, 90, 32, "noise"),
                                         (1920, 1080, 64, "desktop"), (64, 16, 16, "noise")])
def test_gpu_jpeg_matches_cpu(w, h, sh, kind):
    cpu = JpegEncoder(w, h, stripe_height=sh, quality=60, paint_quality=92, paint_over_trigger=2, backend="cpu")
    gpu = JpegEncoder(w, h, stripe_height=sh, quality=60, paint_quality=92, paint_over_trigger=2, backend="hip")
    frames = list(synthetic_frames(w, h, 3, seed=5, kind=kind))
    frames += [frames[-1]] * 3  # static tail -> paint-over on both
    for t, f in enumerate(frames):
        pc, pg = cpu.encode(f, t), gpu.encode(f, t)
        assert [(p.y, p.h) for p in pg] == [(p.y, p.h) for p in pc], f"frame {t}: stripe decisions differ"
        for a, b in zip(pc, pg):
            assert a.data == b.data, f"frame {t} stripe y={a.y}: bytes differ"
            img = Image.open(io.BytesIO(b.data[4:]))
            assert img.size == (w, b.h)
    gpu.request_keyframe()
    assert len(gpu.encode(frames[-1], 99)) == (h + sh - 1) // sh


def test_gpu_jpeg_quality_extremes():
    w, h = 320, 64
    f = next(synthetic_frames(w, h, 1, kind="noise"))
    for q in (1, 100):
        c = JpegEncoder(w, h, stripe_height=64, quality=q, backend="cpu").encode(f, 0)
        g = JpegEncoder(w, h, stripe_height=64, quality=q, backend="hip").encode(f, 0)
        assert [p.data for p in c] == [p.data for p in g]


def test_gpu_capture_session_h264_and_jpeg():
    import pixelflux
    for mode in (1, 0):
        s = pixelflux.default_settings(640, 360, use_cpu=0, source=1, target_fps=60.0, output_mode=mode,
                                       stripe_height=64)
        got, lock = [], threading.Lock()

        def cb(res_ptr, user):
            r = res_ptr.contents
            with lock:
                got.append(bytes(r.data[:r.size]))
        cap = pixelflux.ScreenCapture()
        cap.start_capture(s, pixelflux.StripeCallback(cb))
        time.sleep(1.0)
        st = cap.stats()
        cap.close()
        assert st["frames"] >= 30, st          # paced at 60 fps
        assert st["encode_ms_mean"] < 16.0, st
        assert got
        if mode == 1:
            dec = StripeDecoder(640, 360)
            for p in got:
                dec.feed(p)
        else:
            for p in got[:20]:
                Image.open(io.BytesIO(p[4:])).load()


def test_gpu_server_session():
    import aiohttp
    from selkies_gstreamer_amd.server.data_server import DataStreamingServer
    from selkies_gstreamer_amd.server.settings import Settings

    async def main():
        s = Settings(["--port", "0", "--audio-enabled", "false"], env={})
        srv = DataStreamingServer(s, capture_source="motion")
        port = await srv.start("127.0.0.1", 0)
        async with aiohttp.ClientSession() as sess:
            ws = await sess.ws_connect(f"http://127.0.0.1:{port}/")
            await ws.send_str("SETTINGS," + json.dumps({"initialClientWidth": 1280, "initialClientHeight": 720,
                                                        "encoder": "x264enc-striped", "framerate": 60}))
            dec = StripeDecoder(1280, 720)
            n = 0
            t0 = time.monotonic()
            while n < 60:
                m = await asyncio.wait_for(ws.receive(), 20)
                if isinstance(m.data, bytes):
                    dec.feed(m.data)
                    await ws.send_str(f"CLIENT_FRAME_ACK {int.from_bytes(m.data[2:4], 'big')}")
                    n += 1
            assert time.monotonic() - t0 < 20
            await ws.close()
        await srv.stop()
    asyncio.run(main())


@pytest.mark.parametrize("mode", [2, 3])   # pixelflux OUTPUT_MODE_HEVC / OUTPUT_MODE_AV1
def test_gpu_capture_cbr_hevc_av1_match_cpu(mode):
    """HEVC / AV1 capture sessions (step mode over a pinned pool) under a tight CBR, where
    the controller runs at QP >= 34: the HIP session's packets equal the CPU session's. The
    H.264 front end's automatic deblocking must stay off for them (their own in-loop filters
    make the reference; filtering it again drifted the HIP encoder from the decoder)."""
    import ctypes
    import numpy as np
    import pixelflux
    from selkies_gstreamer_amd.ops.native import PinnedBuffer
    from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
    W, H, N = 320, 192, 24
    src = SyntheticDesktop(W, H, kind="motion", seed=3)
    pool = PinnedBuffer((8, H, W, 4))
    for i in range(8):
        src.frame(i, out=pool.array[i])
    outs = []
    for use_cpu in (1, 0):
        got, lock = [], threading.Lock()

        def cb(res_ptr, n, user):
            with lock:
                got.append(b"".join(bytes(res_ptr[i].data[:res_ptr[i].size]) for i in range(n)))
        s = pixelflux.default_settings(W, H, output_mode=mode, use_paint_over_quality=0, use_cpu=use_cpu,
                                       source=pixelflux.SOURCE_POOL, step_mode=1, pool_frames=8, pool_stride=W * 4,
                                       target_fps=60.0, h264_rc_mode=2, h264_bitrate_kbps=300)
        s.pool = pool.array.ctypes.data
        cap = pixelflux.ScreenCapture()
        thunk = pixelflux.FrameCallback(cb)
        cap.start_frame_capture(s, thunk)
        cap.run(N)
        assert cap.wait(120_000) == 0
        cap.close()
        outs.append(got)
    cpu, gpu = outs
    assert len(cpu) == len(gpu) == N
    for t, (a, b) in enumerate(zip(cpu, gpu)):
        assert a == b, f"frame {t}: HIP capture packets differ from the CPU session's"
