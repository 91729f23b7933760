"""Session host (parallel/multi.py): several complete servers in one process and
one event loop, each with its own port, capture session and encoder; both stream
stripes to their own websocket client at once and stop together."""
import asyncio
import json
import socket

import aiohttp

from selkies_gstreamer_amd.parallel.multi import host, session_argvs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_session_argvs_replace_port():
    out = session_argvs([9001, 9002], ["--port", "1", "--use-cpu", "true"])
    assert out == [["--port", "9001", "--use-cpu", "true"], ["--port", "9002", "--use-cpu", "true"]]


async def _client(port, w, h):
    async with aiohttp.ClientSession() as sess:
        async with sess.ws_connect(f"http://127.0.0.1:{port}/websocket") as ws:
            sent = False
            while True:
                msg = await asyncio.wait_for(ws.receive(), 30)
                if msg.type == aiohttp.WSMsgType.TEXT and "server_settings" in msg.data and not sent:
                    await ws.send_str("SETTINGS," + json.dumps({"initialClientWidth": w, "initialClientHeight": h,
                                                                 "framerate": 30, "encoder": "x264enc-striped"}))
                    sent = True
                elif msg.type == aiohttp.WSMsgType.BINARY and msg.data[0] == 0x04:
                    return (msg.data[6] << 8 | msg.data[7], msg.data[8] << 8 | msg.data[9])


def test_two_sessions_one_process():
    async def main():
        ports = [_free_port(), _free_port()]
        up = []
        stop = asyncio.Event()
        task = asyncio.create_task(host(ports, ["--host", "127.0.0.1", "--use-cpu", "true", "--capture-source",
                                                "synthetic", "--audio-enabled", "false", "--gamepad-enabled",
                                                "false"], stop=stop, ready=lambda srv, port: up.append(port)))
        for _ in range(200):
            if len(up) == 2:
                break
            await asyncio.sleep(0.05)
        assert sorted(up) == sorted(ports)
        sizes = await asyncio.gather(_client(ports[0], 256, 128), _client(ports[1], 320, 192))
        assert sizes[0][0] == 256 and sizes[1][0] == 320     # each session encodes its own stream size
        stop.set()
        await asyncio.wait_for(task, 30)
    asyncio.run(asyncio.wait_for(main(), 90))


def test_launcher_groups_sessions_into_hosts():
    from selkies_gstreamer_amd.parallel.launcher import group_hosts, plan_sessions
    specs = plan_sessions(10, 2, 8082, 20, extra=["--capture-source", "synthetic"])
    hosts = group_hosts(specs, 4)
    assert sorted(p for h in hosts for p in h.all_ports()) == list(range(8082, 8092))
    assert [len(h.all_ports()) for h in hosts] == [4, 1, 4, 1]
    assert all(len({specs[p - 8082].gpu for p in h.all_ports()}) == 1 for h in hosts)   # a host stays on one GPU
    cmd = hosts[0].command("python")
    assert cmd[:3] == ["python", "-m", "selkies_gstreamer_amd.parallel.multi"]
    assert cmd[cmd.index("--") + 1:][:2] == ["--gpu-id", str(hosts[0].gpu)]
    assert group_hosts(specs, 1) is specs


def test_session_argvs_give_each_session_its_display():
    out = session_argvs([9001, 9002], ["--display", ":0", "--use-cpu", "true"], [":20", ":21"])
    assert out == [["--port", "9001", "--display", ":20", "--use-cpu", "true"],
                   ["--port", "9002", "--display", ":21", "--use-cpu", "true"]]


def test_two_displays_stay_separate(monkeypatch):
    """Every session of a host captures, injects into and reconfigures its own X
    display; the process-wide DISPLAY is never consulted or rewritten."""
    from selkies_gstreamer_amd.server.data_server import DisplayState
    from selkies_gstreamer_amd.server.settings import Settings
    monkeypatch.setenv("DISPLAY", ":99")

    async def main():
        ports = [_free_port(), _free_port()]
        servers = {}
        stop = asyncio.Event()
        task = asyncio.create_task(host(ports, ["--host", "127.0.0.1", "--use-cpu", "true", "--capture-source",
                                                "synthetic", "--audio-enabled", "false", "--gamepad-enabled",
                                                "false"], displays=[":20", ":21"], stop=stop,
                                        ready=lambda srv, port: servers.__setitem__(port, srv)))
        for _ in range(200):
            if len(servers) == 2:
                break
            await asyncio.sleep(0.05)
        import os
        assert os.environ["DISPLAY"] == ":99"
        for port, want in zip(ports, (":20", ":21")):
            srv = servers[port]
            assert srv.x_display == want
            assert srv.display_manager.display == want
            st = DisplayState(client=None)
            st.params = dict(Settings([]).client_defaults()) if hasattr(Settings([]), "client_defaults") else {}
            st.params.update({"encoder": "jpeg", "jpeg_quality": 40, "paint_over_jpeg_quality": 90,
                              "use_paint_over_quality": True, "use_cpu": True, "framerate": 30})
            srv.displays["primary"] = st
            cs, _ = srv.capture_settings("primary", 256, 128, 0, 0)
            assert cs.display == want.encode()
        stop.set()
        await asyncio.wait_for(task, 30)
    asyncio.run(asyncio.wait_for(main(), 90))


def test_clipboard_and_xrandr_use_explicit_display(monkeypatch):
    from selkies_gstreamer_amd.server.display import XrandrDisplay, display_env
    from selkies_gstreamer_amd.server.input import Clipboard
    monkeypatch.setenv("DISPLAY", ":99")
    assert Clipboard(":21").env["DISPLAY"] == ":21"
    assert XrandrDisplay(":22").env["DISPLAY"] == ":22"
    assert display_env(None) is None
    assert display_env(":5", {"A": "1"}) == {"A": "1", "DISPLAY": ":5"}
