"""Deployment artefacts: shell scripts parse, configs reference real entry
points, the echo app (reference web.py) echoes, and the TURN REST CLI serves
HMAC credentials."""
import asyncio
import configparser
import subprocess
import sys
from pathlib import Path

import aiohttp
from aiohttp import web

ROOT = Path(__file__).resolve().parents[1]


def test_shell_scripts_parse():
    for p in [ROOT / "deploy/entrypoint.sh", *sorted((ROOT / "deploy/coturn").glob("*.sh"))]:
        r = subprocess.run(["bash", "-n", str(p)], capture_output=True, text=True)
        assert r.returncode == 0, f"{p}: {r.stderr}"


def test_supervisord_programs():
    cp = configparser.ConfigParser(interpolation=None)
    cp.read(ROOT / "deploy/supervisord.conf")
    progs = {s.split(":", 1)[1] for s in cp.sections() if s.startswith("program:")}
    assert {"xvfb", "pulseaudio", "desktop", "selkies", "nginx"} <= progs
    assert "MIT-SHM" in cp["program:xvfb"]["command"] and "XTEST" in cp["program:xvfb"]["command"]


def test_entry_points_exist():
    txt = (ROOT / "deploy/entrypoint.sh").read_text()
    assert "python3 -m selkies_gstreamer_amd webrtc" in txt
    r = subprocess.run([sys.executable, "-m", "selkies_gstreamer_amd.legacy.webrtc_app", "--help"],
                       capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert r.returncode == 0 and "--video_bitrate" in r.stdout
    r = subprocess.run([sys.executable, "-m", "selkies_gstreamer_amd.server.turn", "--help"],
                       capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert r.returncode == 0


def test_echo_app():
    sys.path.insert(0, str(ROOT / "tools"))
    import echo_web

    async def main():
        runner = web.AppRunner(echo_web.make_app())
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        async with aiohttp.ClientSession() as s:
            async with s.ws_connect(f"http://127.0.0.1:{port}/ws") as ws:
                await ws.send_str("ping")
                assert (await ws.receive()).data == "ping"
            async with s.get(f"http://127.0.0.1:{port}/") as r:
                assert "WebSocket" in await r.text()
        await runner.cleanup()
    asyncio.run(main())
