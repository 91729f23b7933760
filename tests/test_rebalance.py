"""Live rebalancing of sessions between GPUs (parallel/rebalance.py, the server's
/api/placement + /api/move, csrc/runtime/capture.cpp CaptureSession::move_to).

CPU tier: the placement policy, the poll loop with fake servers (stall detection,
evacuation, relocation of a session whose GPU stopped answering), the server's
control endpoints against a live server (loopback-only, a CPU session refuses to
move) and the launcher's relocate. GPU tier: a running HIP capture session moved
between frames continues its stream byte-identical to a session that never moved
(P frames, no key frame), for H.264, HEVC and AV1."""
import asyncio
import ctypes
import threading

import aiohttp
import pytest

from selkies_gstreamer_amd.parallel.rebalance import DisplayLoad, Rebalancer, parse_placement, plan_moves


def _d(port, gpu, w=1.0, ms=5.0, frames=100, fps=60.0, disp="primary"):
    return DisplayLoad(f"s{port}", port, disp, gpu, w, ms, frames, fps)


def test_overload_moves_one_display_to_the_lightest_gpu():
    loads = [_d(1, 0, 1.0), _d(2, 0, 1.0, ms=14.0), _d(3, 0, 2.0), _d(4, 1, 1.0)]
    moves = plan_moves(loads, [0, 1, 2], capacity=8)
    assert len(moves) == 1
    d, t = moves[0]
    assert d.gpu == 0 and t == 2          # empty GPU 2 takes it
    # nothing late and under capacity: no move
    assert plan_moves([_d(1, 0, 3.0), _d(2, 1, 1.0)], [0, 1], capacity=8) == []


def test_no_ping_pong():
    # weights 2.0 vs 1.5: the gap (0.5) is below the display's weight, so moving would
    # only swap which GPU is heavier: nothing moves even though the display is late
    assert plan_moves([_d(1, 0, 2.0, ms=20.0), _d(2, 1, 1.5)], [0, 1], capacity=8) == []
    loads = [_d(1, 0, 1.0, ms=20.0), _d(2, 0, 1.0), _d(3, 0, 1.0), _d(4, 1, 0.5)]
    moves = plan_moves(loads, [0, 1], capacity=8)
    assert len(moves) == 1 and moves[0][1] == 1
    # after the move the other GPU is not overloaded by the same rule
    d = moves[0][0]
    after = [x if x is not d else _d(d.port, 1, d.weight, ms=20.0) for x in loads]
    assert plan_moves(after, [0, 1], capacity=8) == []


def test_capacity_and_failed_gpu_evacuation():
    loads = [_d(1, 0, 2.0), _d(2, 0, 1.0), _d(3, 1, 3.0), _d(4, 2, 1.0)]
    moves = plan_moves(loads, [0, 1, 2], capacity=4.5, failed={0})
    assert sorted((m[0].port, m[1]) for m in moves) == [(1, 2), (2, 1)]
    # over capacity (no late display): the heaviest movable display leaves
    moves = plan_moves([_d(1, 0, 3.0), _d(2, 0, 2.0), _d(3, 1, 0.0)], [0, 1], capacity=4.0)
    assert [(m[0].port, m[1]) for m in moves] == [(1, 1)]
    # cooling displays stay
    assert plan_moves([_d(1, 0, 3.0), _d(2, 0, 2.0), _d(3, 1, 0.0)], [0, 1], capacity=4.0,
                      cooling=[(1, "primary"), (2, "primary")]) == []


def test_parse_placement():
    doc = {"gpu_id": 0, "displays": {"primary": {"gpu": 3, "encode_ms_mean": 2.5, "frames": 7, "fps": 30.0,
                                                 "width": 3840, "height": 2160},
                                     "display2": {"gpu": None}}}
    (d,) = parse_placement("s0", 8082, doc)
    assert (d.gpu, d.frames, d.fps) == (3, 7, 30.0) and abs(d.weight - 2.0) < 1e-9


def test_rebalancer_detects_a_stalled_gpu_and_relocates_what_cannot_move():
    state = {8000: {"gpu": 0, "frames": 10}, 8001: {"gpu": 0, "frames": 10}, 8002: {"gpu": 1, "frames": 10}}
    moved, relocated = [], []

    async def fetch(port):
        s = state[port]
        return {"displays": {"primary": {"gpu": s["gpu"], "encode_ms_mean": 3.0, "frames": s["frames"],
                                         "fps": 60.0, "width": 1920, "height": 1080}}}

    async def move(port, display, gpu):
        moved.append((port, gpu))
        if port == 8001:
            return None                      # its GPU does not answer any more
        state[port]["gpu"] = gpu
        return "continued"

    async def relocate(name, gpu):
        relocated.append((name, gpu))

    rb = Rebalancer({"a": [8000], "b": [8001], "c": [8002]}, [0, 1, 2], capacity=8, fetch=fetch, move=move,
                    on_failed_move=relocate)

    async def main():
        assert await rb.step() == []         # first poll: baseline frame counts
        for s in state.values():
            s["frames"] += 5
        assert await rb.step() == []         # everything advances: nothing to do
        state[8002]["frames"] += 5           # GPU 0 stalls (its displays make no frames)
        done = await rb.step()
        assert sorted((d.port, t) for d, t, _ in done) == [(8000, 2), (8001, 1)] or \
            sorted((d.port, t) for d, t, _ in done) == [(8000, 1), (8001, 2)]
        assert relocated and relocated[0][0] == "b"
    asyncio.run(main())


def test_stall_check_treats_a_frame_count_reset_as_alive():
    """A display whose capture was recreated (resize, restart) counts from 0 again: the
    lower count is a new baseline, its GPU is alive and nothing is evacuated."""
    state = {"frames": 500}
    moves = []

    async def fetch(port):
        return {"displays": {"primary": {"gpu": 0, "encode_ms_mean": 3.0, "frames": state["frames"],
                                         "fps": 60.0, "width": 1920, "height": 1080}}}

    async def move(port, display, gpu):
        moves.append(gpu)
        return "continued"
    rb = Rebalancer({"a": [8000]}, [0, 1], capacity=8, fetch=fetch, move=move)

    async def main():
        await rb.step()
        state["frames"] = 3            # capture recreated: counts restart
        assert rb.stalled_gpus(await rb.snapshot()) == set()
        state["frames"] = 9            # and it advances from the new baseline
        assert await rb.step() == []
        assert rb.stalled_gpus(await rb.snapshot()) == {0}   # a real stall still shows
    asyncio.run(main())
    assert moves == []


def test_failed_moves_relocate_a_session_once_per_poll():
    """Two displays of one session host on a stalled GPU, planned onto different GPUs and
    both unmovable: the session is restarted once, on the first target."""
    state = {"frames": 10}
    relocated = []

    async def fetch(port):
        d = {"gpu": 0, "encode_ms_mean": 3.0, "frames": state["frames"], "fps": 60.0, "width": 1920, "height": 1080}
        return {"displays": {"primary": dict(d), "display2": dict(d)}}

    async def move(port, display, gpu):
        return None

    async def relocate(name, gpu):
        relocated.append((name, gpu))
    rb = Rebalancer({"h": [8000]}, [0, 1, 2], capacity=8, fetch=fetch, move=move, on_failed_move=relocate)

    async def main():
        await rb.step()
        done = await rb.step()           # no frames since: GPU 0 stalled
        assert len(done) == 2 and len({t for _, t, _ in done}) == 2
    asyncio.run(main())
    assert len(relocated) == 1 and relocated[0][0] == "h"


def test_control_api_requires_the_token_and_a_direct_caller(tmp_path):
    """The control API answers the launcher's token only: no token configured = off,
    a wrong or missing token or a proxied request (X-Forwarded-For) = 403. With basic
    auth on, the Rebalancer's token requests still get through (no viewer password)."""
    from selkies_gstreamer_amd.parallel.rebalance import http_fetch
    from selkies_gstreamer_amd.server.data_server import DataStreamingServer
    from selkies_gstreamer_amd.server.settings import Settings

    async def main():
        for token, auth in ((None, None), ("t0k", ("u", "pw"))):
            srv = DataStreamingServer(Settings(["--port", "0", "--use-cpu", "true", "--audio-enabled", "false"], env={}),
                                      capture_source="synthetic", control_token=token or "",
                                      basic_auth=auth)
            port = await srv.start("127.0.0.1", 0)
            try:
                async with aiohttp.ClientSession() as sess:
                    hdr = {"X-Selkies-Control-Token": token or "x"}
                    async with sess.get(f"http://127.0.0.1:{port}/api/placement", headers=hdr) as r:
                        assert r.status == (200 if token else 403)
                    if token:
                        async with sess.get(f"http://127.0.0.1:{port}/api/placement",
                                            headers={"X-Selkies-Control-Token": "nope"}) as r:
                            assert r.status == 403
                        async with sess.get(f"http://127.0.0.1:{port}/api/placement",
                                            headers={**hdr, "X-Forwarded-For": "10.0.0.9"}) as r:
                            assert r.status == 403
                        async with sess.post(f"http://127.0.0.1:{port}/api/move", params={"gpu": "1"}) as r:
                            assert r.status == 403
                        # the viewers' routes keep basic auth
                        async with sess.get(f"http://127.0.0.1:{port}/") as r:
                            assert r.status == 401
                        assert (await http_fetch(port, token))["displays"] == {}
                        assert await http_fetch(port, None) is None
            finally:
                await srv.stop()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_server_control_endpoints(tmp_path, monkeypatch):
    """/api/placement lists the running display; /api/move hands the move to the capture
    module (a CPU session cannot move: 409) and pins later restarts to the new GPU."""
    from tests.test_server_e2e import _server, _settings, _recv_until
    monkeypatch.setenv("SELKIES_CONTROL_TOKEN", "tok")
    H = {"X-Selkies-Control-Token": "tok"}

    async def main():
        srv, port, _ = await _server(tmp_path)
        async with aiohttp.ClientSession(headers=H) as sess:
            async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket") as ws:
                await ws.send_str(_settings())
                await _recv_until(ws, lambda m: isinstance(m, bytes))
                # the native frame counter moves after the packet callback: poll briefly
                for _ in range(50):
                    async with sess.get(f"http://127.0.0.1:{port}/api/placement") as r:
                        doc = await r.json()
                    d = doc["displays"]["primary"]
                    if d["frames"] >= 1:
                        break
                    await asyncio.sleep(0.1)
                assert d["width"] == 256 and d["height"] == 128 and d["frames"] >= 1
                async with sess.post(f"http://127.0.0.1:{port}/api/move", params={"gpu": "1"}) as r:
                    assert r.status == 409 and "CPU" in (await r.json())["error"]
                async with sess.post(f"http://127.0.0.1:{port}/api/move", params={"gpu": "x"}) as r:
                    assert r.status == 400
                async with sess.post(f"http://127.0.0.1:{port}/api/move",
                                     params={"gpu": "1", "display": "nope"}) as r:
                    assert r.status == 404
                # a module that moves: the display is pinned to the new GPU
                cap = srv.captures["primary"]
                real = cap.module

                class Movable:
                    device = 0

                    def __getattr__(self, k):
                        return getattr(real, k)

                    def move_to(self, gpu, timeout_ms=10000):
                        self.device = gpu
                        return "continued"
                cap.module = Movable()
                async with sess.post(f"http://127.0.0.1:{port}/api/move", params={"gpu": "3"}) as r:
                    assert (await r.json())["result"] == "continued"
                assert srv._gpu_of["primary"] == 3
                assert srv.placement()["primary"]["gpu"] == 3
                cs, _ = srv.capture_settings("primary", 256, 128, 0, 0)
                assert cs.device == 3
                cap.module = real
        await srv.stop()
    asyncio.run(asyncio.wait_for(main(), 60))


def test_launcher_relocate_restarts_on_the_new_gpu():
    from selkies_gstreamer_amd.parallel.launcher import SessionSpec, Supervisor

    class Proc:
        returncode = None
        terminated = False

        def terminate(self):
            self.terminated = True
    spec = SessionSpec("s0", ":20", 8082, 0)
    others = [SessionSpec(f"o{i}", f":{30 + i}", 9000 + i, 5) for i in range(5)]
    sup = Supervisor([spec, *others], check_health=False)
    sup.procs["s0"] = p = Proc()
    asyncio.run(sup.relocate("s0", 5))
    assert spec.gpu == 5 and p.terminated
    assert spec.hw_queues == 2            # six processes on GPU 5 now: queues resized
    assert spec.env(control_token=sup.control_token)["SELKIES_CONTROL_TOKEN"] == sup.control_token
    assert "--gpu-id" in spec.command() and spec.command()[spec.command().index("--gpu-id") + 1] == "5"


def _capture_run(mode, move_after=None, frames=8, W=256, H=128):
    import pixelflux
    from tests.test_capture_pipeline import _pool
    pool = _pool(W, H)
    got, lock = [], threading.Lock()

    def on_frame(res, n, user):
        with lock:
            got.append([ctypes.string_at(res[i].data, res[i].size) for i in range(n)])
    s = pixelflux.default_settings(W, H, use_cpu=0, source=pixelflux.SOURCE_POOL, step_mode=1, pool_frames=4,
                                   pool_stride=W * 4, stripe_height=64, use_paint_over_quality=0,
                                   output_mode=mode, h264_fullframe=int(mode != 1))
    s.pool = pool.array.ctypes.data
    cap = pixelflux.ScreenCapture()
    cb = pixelflux.FrameCallback(on_frame)
    cap.start_frame_capture(s, cb)
    res = None
    if move_after is None:
        cap.run(frames)
        assert cap.wait(120_000) == 0
    else:
        cap.run(move_after)
        assert cap.wait(120_000) == 0
        res = cap.move_to(0)     # one GPU on the box: a fresh encoder on the same device
        assert cap.device == 0
        cap.run(frames - move_after)
        assert cap.wait(120_000) == 0
        # the capture thread only swaps state and encoders between two frames: the target's
        # build and the old encoder's teardown run on move_to's thread (profiles/r6_move_stall.md)
        assert cap.stats()["move_stall_ms"] < 10.0
    cap.close()
    return got, res


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_hip_capture_moves_between_frames_without_keyframe(mode, capfd):
    from selkies_gstreamer_amd.ops.native import require_gpu
    require_gpu()
    ref, _ = _capture_run(mode)
    got, res = _capture_run(mode, move_after=4)
    assert res == "continued", capfd.readouterr().err[-2000:]   # capture.cpp says why the state was not carried
    assert got == ref
    assert not any(p[1] == 1 for fr in got[4:] for p in fr)   # no key frame after the move


def test_cpu_capture_refuses_to_move():
    import pixelflux
    from tests.test_capture_pipeline import _pool
    pool = _pool(128, 64)
    s = pixelflux.default_settings(128, 64, use_cpu=1, source=pixelflux.SOURCE_POOL, step_mode=1, pool_frames=4,
                                   pool_stride=128 * 4, stripe_height=64)
    s.pool = pool.array.ctypes.data
    cap = pixelflux.ScreenCapture()
    cb = pixelflux.FrameCallback(lambda res, n, user: None)
    cap.start_frame_capture(s, cb)
    try:
        assert cap.device == -1
        with pytest.raises(RuntimeError, match="CPU session"):
            cap.move_to(0, 5000)
    finally:
        cap.close()
