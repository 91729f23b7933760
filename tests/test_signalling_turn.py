"""Legacy signalling server/client (HELLO / SESSION / ROOM relay, health, /turn,
basic auth, static files) and TURN credential generation."""
import asyncio
import base64
import hashlib
import hmac
import json

import aiohttp
import pytest

from selkies_gstreamer_amd.legacy.signalling import SignallingServer
from selkies_gstreamer_amd.legacy.signalling_client import SignallingClient
from selkies_gstreamer_amd.server.turn import (RTCConfigMonitor, hmac_credentials, legacy_rtc_config,
                                               parse_rtc_config, rtc_config, turn_rest_handler)


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


def test_rtc_config_hmac():
    cfg = rtc_config("turn.example.com", 3478, "s3cret", "al:ice", "tcp", True, now=1000)
    turn = cfg["iceServers"][1]
    assert turn["username"] == f"{1000 + 86400}:al-ice"
    expect = base64.b64encode(hmac.new(b"s3cret", turn["username"].encode(), hashlib.sha1).digest()).decode()
    assert turn["credential"] == expect
    assert turn["urls"] == ["turns:turn.example.com:3478?transport=tcp"]
    assert cfg["iceServers"][0]["urls"] == ["stun:turn.example.com:3478", "stun:stun.l.google.com:19302"]
    assert cfg["lifetimeDuration"] == "86400s"
    stun, turns, _ = parse_rtc_config(json.dumps(cfg))
    assert stun[0] == "stun:turn.example.com:3478" and turns[0].startswith("turns://")
    lg = legacy_rtc_config("h", 5349, "u", "p", stun_host="s", stun_port=19302)
    assert lg["iceServers"][0]["urls"][0] == "stun:s:19302" and lg["iceServers"][1]["credential"] == "p"
    with pytest.raises(ValueError):
        parse_rtc_config("{}")


def test_turn_rest_service():
    from aiohttp import web

    async def main():
        app = web.Application()
        defaults = {"secret": "x", "host": "t.example", "port": "443", "stun_host": "t.example", "stun_port": "443",
                    "protocol": "udp", "tls": False}
        app.router.add_route("*", "/", lambda r: turn_rest_handler(r, defaults))
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        async with aiohttp.ClientSession() as s:
            async with s.get(f"http://127.0.0.1:{port}/?username=Bob&protocol=tcp") as r:
                cfg = json.loads(await r.text())
            async with s.post(f"http://127.0.0.1:{port}/", headers={"x-turn-tls": "true"}) as r:
                cfg2 = json.loads(await r.text())
        await runner.cleanup()
        assert cfg["iceServers"][1]["username"].endswith(":bob")
        assert cfg["iceServers"][1]["urls"] == ["turn:t.example:443?transport=tcp"]
        assert cfg2["iceServers"][1]["urls"][0].startswith("turns:")
    run(main())


def test_signalling_session_relay_and_rooms(tmp_path):
    (tmp_path / "index.html").write_text("<html>x</html>")

    async def main():
        srv = SignallingServer(addr="127.0.0.1", port=0, web_root=str(tmp_path), turn_shared_secret="sec",
                               turn_host="t", turn_port="3478")
        port = await srv.start()
        url = f"http://127.0.0.1:{port}/ws"
        # server side application peer (id 1) with metadata, browser peer (id 2)
        app_peer = SignallingClient(url, 1, meta={"res": "1920x1080"})
        browser = SignallingClient(url, 2)
        got = {"sdp": None, "ice": None, "meta": None, "errors": []}
        app_peer.on_sdp = lambda t, sdp: got.__setitem__("sdp", (t, sdp))
        browser.on_ice = lambda i, c: got.__setitem__("ice", (i, c))
        browser.on_session = lambda meta: got.__setitem__("meta", meta)
        browser.on_error = lambda e: got["errors"].append(str(e))
        await app_peer.connect()
        await browser.connect()
        t1 = asyncio.create_task(app_peer.start())
        t2 = asyncio.create_task(browser.start())
        await asyncio.sleep(0.1)
        await browser.setup_call(99)              # unknown peer -> ERROR
        await browser.setup_call(1)
        await asyncio.sleep(0.1)
        await browser.send_sdp("offer", "v=0...")
        await app_peer.send_ice(0, "candidate:1 1 UDP 1 1.2.3.4 5 typ host")
        await asyncio.sleep(0.2)
        assert got["meta"] == {"res": "1920x1080"}
        assert got["sdp"] == ("offer", "v=0...") and got["ice"][0] == 0
        assert any("not found" in e for e in got["errors"])
        await browser.stop()
        await asyncio.sleep(0.2)
        assert not srv.sessions and 1 not in srv.peers   # the session partner is reset too
        await app_peer.stop()
        for t in (t1, t2):
            t.cancel()
        # rooms
        async with aiohttp.ClientSession() as s:
            a = await s.ws_connect(url)
            b = await s.ws_connect(url)
            await a.send_str("HELLO alice")
            await b.send_str("HELLO bob")
            assert (await a.receive()).data == "HELLO" and (await b.receive()).data == "HELLO"
            await a.send_str("ROOM r1")
            assert (await a.receive()).data == "ROOM_OK "
            await b.send_str("ROOM r1")
            assert (await b.receive()).data == "ROOM_OK alice"
            assert (await a.receive()).data == "ROOM_PEER_JOINED bob"
            await b.send_str("ROOM_PEER_MSG alice hi there")
            assert (await a.receive()).data == "ROOM_PEER_MSG bob hi there"
            await b.close()
            assert (await a.receive()).data == "ROOM_PEER_LEFT bob"
            dup = await s.ws_connect(url)
            await dup.send_str("HELLO alice")           # duplicate uid -> closed
            m = await dup.receive()
            assert m.type == aiohttp.WSMsgType.CLOSE
            await a.close()
            async with s.get(f"http://127.0.0.1:{port}/health") as r:
                assert r.status == 200 and (await r.text()) == "OK\n"
            async with s.get(f"http://127.0.0.1:{port}/turn", headers={"x-auth-user": "carol"}) as r:
                assert (await r.json())["iceServers"][1]["username"].endswith(":carol")
            async with s.get(f"http://127.0.0.1:{port}/") as r:
                assert "x" in await r.text()
            async with s.get(f"http://127.0.0.1:{port}/../../etc/passwd") as r:
                assert r.status == 404
        await srv.stop()
    run(main())


def test_signalling_basic_auth():
    async def main():
        srv = SignallingServer(addr="127.0.0.1", port=0, enable_basic_auth=True, basic_auth_user="u",
                               basic_auth_password="p")
        port = await srv.start()
        async with aiohttp.ClientSession() as s:
            async with s.get(f"http://127.0.0.1:{port}/health") as r:
                assert r.status == 401 and "WWW-Authenticate" in r.headers
        async with aiohttp.ClientSession(auth=aiohttp.BasicAuth("u", "p")) as s:
            async with s.get(f"http://127.0.0.1:{port}/health") as r:
                assert r.status == 200
        await srv.stop()
    run(main())


def test_rtc_config_monitor(tmp_path):
    async def main():
        seen = []
        f = tmp_path / "rtc.json"
        f.write_text(json.dumps(rtc_config("h", 1, "s", "u", now=0)))
        mon = RTCConfigMonitor(lambda cfg: seen.append(cfg), json_file=str(f))
        assert await mon.refresh() and not await mon.refresh()
        hm = RTCConfigMonitor(lambda cfg: seen.append(cfg), hmac_params={"host": "h", "port": 1, "secret": "s"})
        assert await hm.refresh()
        assert len(seen) == 2
    run(main())
