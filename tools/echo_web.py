"""WebSocket echo + static demo page (reference web.py:1-30 + static/index.html,
SURVEY C47): a connectivity check for proxies / TURN-less networks that is
independent of the streaming stack.

    python tools/echo_web.py --port 8090
"""
import argparse

from aiohttp import WSMsgType, web

PAGE = """<!DOCTYPE html><meta charset=utf-8><title>echo</title>
<pre id=log></pre><script>
const ws = new WebSocket((location.protocol === 'https:' ? 'wss://' : 'ws://') + location.host + '/ws');
const log = (m) => document.getElementById('log').textContent += m + '\\n';
ws.onopen = () => { log('open'); ws.send('hello ' + Date.now()); };
ws.onmessage = (e) => log('echo: ' + e.data);
ws.onclose = () => log('closed');
</script>"""


async def ws_handler(request):
    ws = web.WebSocketResponse()
    await ws.prepare(request)
    async for msg in ws:
        if msg.type == WSMsgType.TEXT:
            await ws.send_str(msg.data)
        elif msg.type == WSMsgType.BINARY:
            await ws.send_bytes(msg.data)
    return ws


def make_app() -> web.Application:
    app = web.Application()
    app.router.add_get("/ws", ws_handler)
    app.router.add_get("/", lambda r: web.Response(text=PAGE, content_type="text/html"))
    return app


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=8090)
    web.run_app(make_app(), port=ap.parse_args().port)
