"""Pure server logic: settings precedence, protocol helpers, backpressure with a
fake clock, upload path sanitising, layout/modelines, gamepad ABI, input mapping.

Reference parity notes: the reference has no tests for these; the
expected values below come from its behavior (selkies.py / settings.py /
input_handler.py line refs in the module docstrings) and, for CVT, from the
``cvt`` utility's published modelines.
"""
import asyncio
import base64
import json
import os
import socket
import struct

import pytest

from selkies_gstreamer_amd.server import protocol
from selkies_gstreamer_amd.server.display import compute_layout, cvt_modeline, fit_resolution, parse_xrandr
from selkies_gstreamer_amd.server.gamepad import (JS_CONFIG_SIZE, XPAD, GamepadHub, map_event, pack_input_events,
                                                 pack_js_config, pack_js_event, unpack_js_config)
from selkies_gstreamer_amd.server.input import InputHandler, RecordingInjector, char_to_keysym, keysym_to_char
from selkies_gstreamer_amd.server.settings import Settings, build_specs


# ----------------------------------------------------------------------------- settings
def test_settings_count_and_defaults():
    specs = build_specs()
    # the reference's 56 + H.264 quality tools (AQ, quarter-pel, Intra4x4) + ui_dashboard + h264_bitrate (K10 CBR)
    assert len(specs) == 61
    s = Settings([], env={})
    assert s.h264_aq_strength == 0 and s.h264_subpel == (True, False) and s.h264_intra4x4 == (False, False)
    assert s.encoder == "x264enc" and s.framerate == (8, 120) and s.port == 8082
    assert s.audio_enabled == (True, False)
    assert s.file_transfers == ["upload", "download"]
    assert s.initial("framerate") == 60 and s.initial("h264_crf") == 25 and s.initial("jpeg_quality") == 40
    assert s.initial("h264_bitrate") == 0      # CRF unless a bitrate is set


def test_settings_precedence_cli_env_legacy():
    env = {"SELKIES_PORT": "9000", "CUSTOM_WS_PORT": "9100", "SELKIES_ENCODER": "jpeg,x264enc"}
    s = Settings(["--port", "9200"], env=env)
    assert s.port == 9200
    s = Settings([], env=env)
    assert s.port == 9000 and s.encoder == "jpeg"
    assert s.by_name["encoder"].allowed == ["jpeg", "x264enc"]
    s = Settings([], env={"CUSTOM_WS_PORT": "9100"})
    assert s.port == 9100


def test_settings_bool_lock_range_and_unknown_flags():
    s = Settings(["--use-cpu", "true|locked", "--framerate", "30", "--h264-crf", "10-20", "--bogus-legacy", "x"],
                 env={})
    assert s.use_cpu == (True, True)
    assert s.framerate == (30, 30) and s.initial("framerate") == 30
    assert s.h264_crf == (10, 20)
    assert s.unknown_args == ["--bogus-legacy", "x"]
    # sanitize: clamp ranges, locked bools ignore the client, invalid enum -> first allowed
    assert s.sanitize("h264_crf", 45) == 20 and s.sanitize("h264_crf", 3) == 10
    assert s.sanitize("use_cpu", "false") is True
    assert s.sanitize("encoder", "vp9") == "x264enc"
    assert s.sanitize("framerate", None) == 30


def test_settings_manual_resolution_autolock():
    s = Settings(["--manual-width", "1280"], env={})
    assert s.is_manual_resolution_mode == (True, True)
    assert s.manual_width == 1280 and s.manual_height == 768


def test_server_settings_payload_shape():
    s = Settings([], env={})
    p = s.client_payload()
    assert p["type"] == "server_settings"
    st = p["settings"]
    assert "port" not in st and "debug" not in st and "watermark_path" not in st
    assert st["framerate"] == {"value": [8, 120], "min": 8, "max": 120, "default": 60} or \
        st["framerate"] == {"value": (8, 120), "min": 8, "max": 120, "default": 60}
    assert st["encoder"]["allowed"] == ["x264enc", "x264enc-striped", "jpeg", "x265enc", "svtav1enc"]
    assert st["audio_enabled"] == {"value": True, "locked": False}
    json.dumps(p)


# ----------------------------------------------------------------------------- protocol
def test_parse_settings_payload_types():
    p = protocol.parse_settings_payload(json.dumps({"framerate": "30", "h264_fullcolor": "true",
                                                    "encoder": "jpeg", "displayId": "display2"}))
    assert p["framerate"] == 30 and p["h264_fullcolor"] is True and p["encoder"] == "jpeg"
    assert p["h264_crf"] is None and p["displayId"] == "display2"
    with pytest.raises(ValueError):
        protocol.parse_settings_payload("[1,2]")


def test_frame_desync_wraps():
    assert protocol.frame_desync(10, 5) == 5
    assert protocol.frame_desync(3, 65534) == 5
    assert protocol.parse_frame_ack("CLIENT_FRAME_ACK 42") == 42


def test_backpressure_fake_clock():
    f = protocol.DisplayFlow()
    t = 100.0
    f.reset(t)
    assert f.evaluate(t, True, 60) is True           # no ACK yet -> lifted
    for i in range(1, 200):
        f.on_sent(i, t)
    f.on_ack(50, t + 0.02)
    assert f.smoothed_rtt_ms == pytest.approx(20.0)
    assert f.evaluate(t + 0.1, True, 60) is False    # 149 frames behind > 120 allowed at 60 fps
    f.on_ack(150, t + 0.2)
    assert f.evaluate(t + 0.3, True, 60) is True     # 49 behind
    # stall: no ACK for > 4 s
    assert f.evaluate(t + 5.0, True, 60) is False
    # capture stopped -> always lifted
    assert f.evaluate(t + 5.1, False, 60) is True
    # RTT compensation: 1 s RTT at 60 fps allows 60 extra frames
    g = protocol.DisplayFlow()
    g.reset(0.0)
    g.on_sent(1, 0.0)
    g.on_ack(1, 1.0)
    for i in range(2, 172):
        g.on_sent(i, 1.0)
    g.on_ack(1, 1.0)
    assert g.evaluate(1.1, True, 60) is True        # 170 behind - 60 adj = 110 <= 120
    # suspicious gap (counter reset) lifts backpressure
    h = protocol.DisplayFlow()
    h.reset(0.0)
    h.on_sent(40000, 0.0)
    h.on_ack(3, 0.0)
    assert h.evaluate(0.1, True, 60) is True


def test_sanitize_upload_path(tmp_path):
    root = str(tmp_path)
    assert protocol.sanitize_upload_path(root, "a/b.txt") == os.path.join(root, "a", "b.txt")
    assert protocol.sanitize_upload_path(root, "/etc/passwd") == os.path.join(root, "etc", "passwd")
    assert protocol.sanitize_upload_path(root, "../x") is None
    assert protocol.sanitize_upload_path(root, "a/../../x") is None
    assert protocol.sanitize_upload_path(root, "") is None
    assert protocol.sanitize_upload_path(root, "./.") is None
    os.symlink("/tmp", os.path.join(root, "link"))
    assert protocol.sanitize_upload_path(root, "link/evil") is None
    assert protocol.parse_upload_start("FILE_UPLOAD_START:dir/a:b.txt:123") == ("dir/a:b.txt", 123)


def test_clipboard_messages_roundtrip():
    small = protocol.clipboard_messages(b"hello")
    assert small == ["clipboard," + base64.b64encode(b"hello").decode()]
    img = protocol.clipboard_messages(b"\x89PNG", "image/png")
    assert img[0].startswith("clipboard_binary,image/png,")
    big = bytes(range(256)) * 10
    parts = protocol.clipboard_messages(big, "text/plain", chunk=1000)
    assert parts[0] == f"clipboard_start,text/plain,{len(big)}" and parts[-1] == "clipboard_finish"
    asm = protocol.ClipboardAssembler()
    asm.start("text/plain", len(big))
    for p in parts[1:-1]:
        assert asm.data(p.split(",", 1)[1])
    assert asm.end() == ("text/plain", big)
    asm.start("text/plain", 5)
    asm.data(base64.b64encode(b"abc").decode())
    assert asm.end() is None


# ----------------------------------------------------------------------------- display
def test_layouts():
    l, w, h = compute_layout({"primary": {"width": 1921, "height": 1080}})
    assert l == {"primary": {"x": 0, "y": 0, "w": 1921, "h": 1080}} and (w, h) == (1928, 1080)
    for pos, exp in {"right": ({"x": 0, "y": 0}, {"x": 1920, "y": 0}, (3200, 1080)),
                     "left": ({"x": 1280, "y": 0}, {"x": 0, "y": 0}, (3200, 1080)),
                     "down": ({"x": 0, "y": 0}, {"x": 0, "y": 1080}, (1920, 1800)),
                     "up": ({"x": 0, "y": 720}, {"x": 0, "y": 0}, (1920, 1800))}.items():
        l, w, h = compute_layout({"primary": {"width": 1920, "height": 1080},
                                  "display2": {"width": 1280, "height": 720, "position": pos}})
        assert {k: l["primary"][k] for k in "xy"} == exp[0]
        assert {k: l["display2"][k] for k in "xy"} == exp[1]
        assert (w, h) == exp[2]
    assert compute_layout({}) == ({}, 0, 0)
    assert fit_resolution(8000, 4500) == (7680, 4320)


def test_cvt_matches_cvt_utility():
    assert cvt_modeline(1920, 1080)[1] == "173.00 1920 2048 2248 2576 1080 1083 1088 1120 -hsync +vsync"
    assert cvt_modeline(1280, 720)[1] == "74.50 1280 1344 1472 1664 720 723 728 748 -hsync +vsync"
    assert cvt_modeline(1024, 768)[1] == "63.50 1024 1072 1176 1328 768 771 775 798 -hsync +vsync"


def test_parse_xrandr():
    text = ("Screen 0: minimum 8 x 8, current 1920 x 1080, maximum 32767 x 32767\n"
            "DUMMY0 connected primary 1920x1080+0+0 0mm x 0mm\n"
            "   1920x1080     60.00*+\n   1280x720      60.00  \n"
            "DUMMY1 disconnected\n   800x600   60.00\n")
    assert parse_xrandr(text) == ("DUMMY0", "1920x1080", ["1280x720", "1920x1080"])


# ----------------------------------------------------------------------------- gamepad
def test_js_config_abi():
    raw = pack_js_config()
    assert len(raw) == JS_CONFIG_SIZE == 1360
    name = raw[:255].split(b"\0", 1)[0]
    assert name == b"Microsoft X-Box 360 pad"
    vendor, product, version, nb, na = struct.unpack_from("<5H", raw, 256)
    assert (vendor, product, version, nb, na) == (0x045E, 0x028E, 0x0114, 11, 8)
    btns = struct.unpack_from("<512H", raw, 266)
    assert btns[:3] == (0x130, 0x131, 0x133) and btns[11] == 0
    axes = raw[266 + 1024: 266 + 1024 + 64]
    assert list(axes[:8]) == [0, 1, 2, 3, 4, 5, 0x10, 0x11]
    assert unpack_js_config(raw).num_btns == 11


def test_gamepad_mapping():
    e = map_event(XPAD, 0, 1.0, True)            # A
    assert (e.js_type, e.js_number, e.js_value, e.ev_code, e.ev_value) == (1, 0, 1, 0x130, 1)
    e = map_event(XPAD, 7, 1.0, True)            # RT button -> RZ axis
    assert (e.js_type, e.js_number, e.ev_code, e.js_value) == (2, 5, 0x05, 32767)
    e = map_event(XPAD, 12, 1.0, True)           # d-pad up -> HAT0Y -1
    assert (e.ev_code, e.ev_value, e.js_value) == (0x11, -1, -32767)
    e = map_event(XPAD, 2, -1.0, False)          # right stick X
    assert (e.js_number, e.ev_code, e.ev_value) == (3, 0x03, -32767)
    assert map_event(XPAD, 99, 1.0, True) is None
    assert len(pack_js_event(e)) == 8
    assert len(pack_input_events(e, 8)) == 48 and len(pack_input_events(e, 4)) == 32


def test_gamepad_socket_roundtrip(tmp_path):
    async def run():
        hub = GamepadHub(str(tmp_path), slots=1)
        await hub.start()
        r, w = await asyncio.open_unix_connection(str(tmp_path / "selkies_js0.sock"))
        cfg = await r.readexactly(1360)
        assert cfg == pack_js_config()
        w.write(bytes([8]))
        await w.drain()
        re_, we = await asyncio.open_unix_connection(str(tmp_path / "selkies_event1000.sock"))
        await re_.readexactly(1360)
        we.write(bytes([8]))
        await we.drain()
        await asyncio.sleep(0.05)
        hub.button(0, 1, 1.0)                    # B
        ev = await asyncio.wait_for(r.readexactly(8), 2)
        _, value, typ, num = struct.unpack("<IhBB", ev)
        assert (value, typ, num) == (1, 1, 1)
        ie = await asyncio.wait_for(re_.readexactly(48), 2)
        _, _, t, code, val = struct.unpack_from("<qqHHi", ie, 0)
        assert (t, code, val) == (1, 0x131, 1)
        w.close()
        we.close()
        await hub.close()
    asyncio.run(run())


# ----------------------------------------------------------------------------- input
def test_keysym_helpers():
    assert keysym_to_char(0x41) == "A" and keysym_to_char(0x010020AC) == "€"
    assert keysym_to_char(0xFF0D) is None
    assert char_to_keysym("a") == 0x61 and char_to_keysym("€") == 0x010020AC and char_to_keysym("\n") == 0xFF0D


def test_input_keys_and_mouse():
    inj = RecordingInjector()
    h = InputHandler(inj, layout_offset=lambda d: (100, 0) if d == "display2" else (0, 0))

    async def run():
        await h.on_message("kd,97")                # 'a' letter -> plain press
        await h.on_message("ku,97")
        await h.on_message("kd,49")                # '1' non-alpha, no modifier -> atomic type
        await h.on_message("ku,49")
        await h.on_message("kd,65507")             # Control_L
        await h.on_message("kd,49")                # with Ctrl -> real key press
        await h.on_message("ku,49")
        await h.on_message("ku,65507")
        await h.on_message("m,10,20,1,0")          # move + left press
        await h.on_message("m,10,20,0,0")          # left release
        await h.on_message("m2,0,0,8,3")           # wheel down x3
        await h.on_message("m2,0,0,0,3")
        await h.on_message("m2,0,0,16,0")          # Forward button -> Alt+Right
        await h.on_message("m2,0,0,0,0")
        await h.on_message("m,5,5,0,0", "display2")  # offset by the display layout
        await h.on_message("co,end,hi")
    asyncio.run(run())
    ev = inj.events
    assert ev[:2] == [("key", 97, True), ("key", 97, False)]
    assert ev[2:4] == [("key", 49, True), ("key", 49, False)]       # typed atomically on kd
    assert ev[4:7] == [("key", 65507, True), ("key", 49, True), ("key", 49, False)]
    assert ("motion", 10, 20) in ev and ("button", 1, True) in ev and ("button", 1, False) in ev
    assert [e for e in ev if e[:2] == ("button", 5)] == [("button", 5, True), ("button", 5, False)] * 3
    i = ev.index(("key", 0xFFE9, True))
    assert ev[i:i + 4] == [("key", 0xFFE9, True), ("key", 0xFF53, True), ("key", 0xFF53, False),
                           ("key", 0xFFE9, False)]
    assert ("motion", 105, 5) in ev
    assert ev[-4:] == [("key", 0x68, True), ("key", 0x68, False), ("key", 0x69, True), ("key", 0x69, False)]


def test_input_gamepad_dispatch(tmp_path):
    async def run():
        hub = GamepadHub(str(tmp_path), slots=4)
        await hub.start()
        h = InputHandler(RecordingInjector(), gamepads=hub)
        await h.on_message("js,c,1," + base64.b64encode(b"Pad").decode() + ",4,17")
        assert hub.pads[1].client_name == "Pad"
        await h.on_message("js,b,1,0,1")
        await h.on_message("js,a,1,0,0.5")
        await h.on_message("js,d,1")
        assert hub.pads[1].client_name is None
        await hub.close()
    asyncio.run(run())


def test_queue_overflow_requests_keyframe_and_skips_p_frames():
    """A full native->loop queue drops an H.264 frame for every viewer: the server
    asks for a keyframe and queues no P frame until it arrives (JPEG just drops)."""
    import asyncio as aio
    from selkies_gstreamer_amd.server.data_server import Capture, DataStreamingServer
    from selkies_gstreamer_amd.server.settings import Settings

    class Mod:
        kf = 0

        def request_keyframe(self):
            Mod.kf += 1

    async def main():
        srv = DataStreamingServer(Settings([]), capture_factory=Mod)
        q = aio.Queue(maxsize=2)
        srv.captures["primary"] = Capture("primary", Mod(), q, None)
        for fid in range(3):                       # third frame overflows
            srv._put_frame("primary", q, ([b"p"], fid == 0, fid, 0), False)
        assert Mod.kf == 1 and q.qsize() == 2
        q.get_nowait()
        q.get_nowait()
        srv._put_frame("primary", q, ([b"p"], False, 3, 0), False)
        assert q.qsize() == 0                      # P frame after the drop is not queued
        srv._put_frame("primary", q, ([b"i"], True, 4, 0), False)
        assert q.qsize() == 1 and "primary" not in srv._resync
        srv._put_frame("primary", q, ([b"p"], False, 5, 0), False)
        assert q.qsize() == 2
        srv._put_frame("primary", q, ([b"j"], False, 6, 0), True)   # JPEG overflow: no keyframe request
        assert Mod.kf == 1 and "primary" not in srv._resync
    aio.run(main())
