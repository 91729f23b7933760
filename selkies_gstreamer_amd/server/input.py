"""Client input -> X11 (keyboard, pointer), gamepads, clipboard, cursor.

Message vocabulary handled (reference input_handler.py:1507-1697):
``kd,<keysym>`` ``ku,<keysym>`` ``kr`` (reset modifiers) ``m,x,y,mask,mag`` /
``m2,dx,dy,mask,mag`` (absolute / relative pointer; mask bits 0-2 = L/M/R, 3 =
wheel down or Back, 4 = wheel up or Forward, 6/7 = wheel left/right) ``p,<0|1>``
``vb,`` ``ab,`` ``js,c|d|b|a,...`` (gamepads) ``cw,<b64>`` ``cb,<mime>,<b64>``
``cws/cbs/cwd/cbd/cwe/cbe`` (multipart clipboard) ``cr`` (clipboard read)
``_arg_fps`` ``_arg_resize`` ``_f`` ``_l`` ``_stats_video/_stats_audio``
``co,end,<text>`` ``pong``.

Injection goes through an :class:`Injector`: :class:`X11Injector` drives XTest
natively (csrc/input/x11_input.cpp, no xdotool/pynput processes),
:class:`UinputMouse` forwards relative motion to a uinput helper socket
(msgpack datagrams, reference ``--uinput_mouse_socket``), and tests use
:class:`RecordingInjector`.
"""
from __future__ import annotations

import asyncio
import base64
import ctypes
import io
import logging
import os
import shutil
import time
from typing import Awaitable, Callable, Optional

from . import protocol
from .gamepad import GamepadHub

log = logging.getLogger("input")

SHIFT_KEYSYMS = {0xFFE1, 0xFFE2}
MODIFIER_KEYSYMS = {0xFFE1, 0xFFE2, 0xFFE3, 0xFFE4, 0xFFE9, 0xFFEA, 0xFE03, 0xFFE7, 0xFFE8, 0xFFEB, 0xFFEC}
RESET_KEYSYMS = (0xFFE3, 0xFFE1, 0xFFE9, 0xFFE4, 0xFFE2, 0xFE03, 0xFFE7, 0xFFE8, 0x66, 0x46, 0x6D, 0x4D, 0xFF1B)
XK_ALT_L, XK_LEFT, XK_RIGHT = 0xFFE9, 0xFF51, 0xFF53

# X core pointer buttons
BTN_LEFT, BTN_MIDDLE, BTN_RIGHT, WHEEL_UP, WHEEL_DOWN, WHEEL_LEFT, WHEEL_RIGHT = 1, 2, 3, 4, 5, 6, 7


def keysym_to_char(keysym: int) -> Optional[str]:
    """Printable character of a keysym (Latin-1 range or the 0x01xxxxxx Unicode plane)."""
    if 0x20 <= keysym <= 0xFF:
        return chr(keysym)
    if keysym & 0xFF000000 == 0x01000000:
        try:
            return chr(keysym & 0x00FFFFFF)
        except ValueError:
            return None
    return None


def char_to_keysym(ch: str) -> int:
    cp = ord(ch)
    if 0x20 <= cp <= 0x7E or 0xA0 <= cp <= 0xFF:
        return cp
    if ch == "\n":
        return 0xFF0D
    if ch == "\t":
        return 0xFF09
    return 0x01000000 | cp


class Injector:
    available = False

    def key(self, keysym: int, down: bool, shift: bool) -> None: ...
    def motion(self, x: int, y: int) -> None: ...
    def motion_rel(self, dx: int, dy: int) -> None: ...
    def button(self, b: int, down: bool) -> None: ...
    def close(self) -> None: ...


class RecordingInjector(Injector):
    available = True

    def __init__(self):
        self.events: list[tuple] = []

    def key(self, keysym, down, shift):
        self.events.append(("key", keysym, down))

    def motion(self, x, y):
        self.events.append(("motion", x, y))

    def motion_rel(self, dx, dy):
        self.events.append(("rel", dx, dy))

    def button(self, b, down):
        self.events.append(("button", b, down))


class X11Injector(Injector):
    def __init__(self, display: Optional[str] = None):
        from selkies_gstreamer_amd.ops import native
        self.L = native.lib()
        L = self.L
        L.sk_x11_input_open.restype = ctypes.c_void_p
        L.sk_x11_input_open.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.sk_x11_input_close.argtypes = [ctypes.c_void_p]
        L.sk_x11_key.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
        L.sk_x11_motion.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.sk_x11_motion_rel.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.sk_x11_button.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        self.h = L.sk_x11_input_open(display.encode() if display else None, 0)
        self.available = bool(self.h)
        if not self.h:
            log.warning("X11 input unavailable: %s", L.sk_last_error().decode())

    def key(self, keysym, down, shift):
        if self.h and self.L.sk_x11_key(self.h, keysym & 0xFFFFFFFF, int(down), int(shift)) != 0:
            log.debug("no keycode for keysym 0x%x", keysym)

    def motion(self, x, y):
        if self.h:
            self.L.sk_x11_motion(self.h, int(x), int(y))

    def motion_rel(self, dx, dy):
        if self.h:
            self.L.sk_x11_motion_rel(self.h, int(dx), int(dy))

    def button(self, b, down):
        if self.h:
            self.L.sk_x11_button(self.h, int(b), int(down))

    def close(self):
        if self.h:
            self.L.sk_x11_input_close(self.h)
            self.h = None


class UinputMouse(Injector):
    """Relative mouse through a uinput helper socket; everything else delegated."""
    EV_KEY, EV_REL = 0x01, 0x02
    BUTTONS = {BTN_LEFT: 0x110, BTN_MIDDLE: 0x112, BTN_RIGHT: 0x111}

    def __init__(self, path: str, inner: Injector):
        import socket
        import msgpack
        self.path, self.inner, self._pack = path, inner, msgpack.packb
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        self.available = inner.available

    def _emit(self, code, value, syn=True):
        data = self._pack({"args": [list(code), value], "kwargs": {"syn": syn}}, use_bin_type=True)
        try:
            self.sock.sendto(data, self.path)
        except OSError as e:
            log.debug("uinput send failed: %s", e)

    def key(self, keysym, down, shift):
        self.inner.key(keysym, down, shift)

    def motion(self, x, y):
        self.inner.motion(x, y)

    def motion_rel(self, dx, dy):
        self._emit((self.EV_REL, 0x00), dx, syn=False)
        self._emit((self.EV_REL, 0x01), dy)

    def button(self, b, down):
        if b in self.BUTTONS:
            self._emit((self.EV_KEY, self.BUTTONS[b]), int(down))
        elif b in (WHEEL_UP, WHEEL_DOWN):
            if down:
                self._emit((self.EV_REL, 0x08), 1 if b == WHEEL_UP else -1)
        else:
            self.inner.button(b, down)


class Clipboard:
    """X clipboard through xclip (or xsel for text); a no-op when neither exists."""
    IMAGE_TYPES = ("image/png", "image/jpeg", "image/bmp", "image/svg", "image/webp")

    def __init__(self, display: Optional[str] = None):
        self.xclip = shutil.which("xclip")
        self.xsel = shutil.which("xsel")
        self.display = display if display is not None else os.environ.get("DISPLAY")
        self.env = dict(os.environ, DISPLAY=self.display) if self.display else None

    @property
    def available(self):
        return bool(self.xclip or self.xsel) and bool(self.display)

    async def _run(self, cmd, data: Optional[bytes] = None, timeout=2.0):
        p = await asyncio.create_subprocess_exec(*cmd, stdin=asyncio.subprocess.PIPE if data is not None else None,
                                                 stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.DEVNULL,
                                                 env=self.env)
        out, _ = await asyncio.wait_for(p.communicate(data), timeout)
        return p.returncode, out

    async def read(self, binary: bool = False):
        if not self.available:
            return None, None
        try:
            if self.xclip:
                rc, out = await self._run([self.xclip, "-selection", "clipboard", "-o", "-t", "TARGETS"])
                if rc != 0:
                    return None, None
                targets = out.decode(errors="replace").split()
                if binary:
                    for mime in self.IMAGE_TYPES:
                        if mime in targets:
                            rc, data = await self._run([self.xclip, "-selection", "clipboard", "-o", "-t", mime])
                            if rc == 0 and data:
                                return data, mime
                if "UTF8_STRING" in targets:
                    rc, data = await self._run([self.xclip, "-selection", "clipboard", "-o", "-t", "UTF8_STRING"])
                    if rc == 0:
                        return data.decode("utf-8", "replace"), "text/plain"
                return None, None
            rc, data = await self._run([self.xsel, "--clipboard", "--output"])
            return (data.decode("utf-8", "replace"), "text/plain") if rc == 0 else (None, None)
        except (OSError, asyncio.TimeoutError):
            return None, None

    async def write(self, data, mime: str = "text/plain") -> bool:
        if not data:
            return True
        if not self.available:
            return False
        raw = data if isinstance(data, bytes) else data.encode()
        try:
            if self.xclip:
                rc, _ = await self._run([self.xclip, "-selection", "clipboard", "-i", "-t", mime], raw)
            elif mime == "text/plain":
                rc, _ = await self._run([self.xsel, "--clipboard", "--input"], raw)
            else:
                return False
            return rc == 0
        except (OSError, asyncio.TimeoutError):
            return False


def cursor_message(serial: int, w: int, h: int, xhot: int, yhot: int, argb, cap: int = 32) -> dict:
    """ARGB32 cursor -> ``cursor,{json}`` payload dict (cropped, scaled to cap, PNG b64)."""
    empty = {"curdata": "", "width": 0, "height": 0, "hotx": 0, "hoty": 0, "handle": serial}
    if w == 0 or h == 0:
        return empty
    from PIL import Image
    import numpy as np
    px = np.asarray(argb, dtype=np.uint32)[: w * h].reshape(h, w)
    bgra = px.view(np.uint8).reshape(h, w, 4)  # little endian ARGB32 -> B,G,R,A bytes
    im = Image.frombuffer("RGBA", (w, h), bgra.tobytes(), "raw", "BGRA", 0, 1)
    bbox = im.getbbox()
    if bbox is None:
        return empty
    im = im.crop(bbox)
    hx, hy = xhot - bbox[0], yhot - bbox[1]
    if max(im.width, im.height) > cap:
        s = cap / max(im.width, im.height)
        im = im.resize((max(1, int(im.width * s)), max(1, int(im.height * s))), Image.LANCZOS)
        hx, hy = int(hx * s), int(hy * s)
    buf = io.BytesIO()
    im.save(buf, "PNG")
    return {"curdata": base64.b64encode(buf.getvalue()).decode(), "width": im.width, "height": im.height,
            "hotx": hx, "hoty": hy, "handle": serial}


class CursorWatcher:
    """XFixes cursor-change watcher on its own X connection, run in a thread."""

    def __init__(self, on_cursor: Callable[[dict], None], display: Optional[str] = None, cap: int = 32):
        from selkies_gstreamer_amd.ops import native
        L = self.L = native.lib()
        L.sk_x11_input_open.restype = ctypes.c_void_p
        L.sk_x11_input_open.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.sk_x11_cursor_wait.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.sk_x11_cursor_image.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)] + \
            [ctypes.POINTER(ctypes.c_int)] * 4 + [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
        self.h = L.sk_x11_input_open(display.encode() if display else None, 1)
        self.on_cursor, self.cap = on_cursor, cap
        self.running = False

    @property
    def available(self):
        return bool(self.h)

    def snapshot(self) -> Optional[dict]:
        serial = ctypes.c_uint64()
        w, h, xh, yh = (ctypes.c_int() for _ in range(4))
        buf = (ctypes.c_uint32 * (256 * 256))()
        n = self.L.sk_x11_cursor_image(self.h, ctypes.byref(serial), ctypes.byref(w), ctypes.byref(h),
                                       ctypes.byref(xh), ctypes.byref(yh), buf, len(buf))
        if n < 0:
            return None
        return cursor_message(serial.value, w.value, h.value, xh.value, yh.value, buf, self.cap)

    def run(self):
        self.running = True
        msg = self.snapshot()
        if msg:
            self.on_cursor(msg)
        while self.running:
            if self.L.sk_x11_cursor_wait(self.h, 100) == 1:
                msg = self.snapshot()
                if msg:
                    self.on_cursor(msg)

    def stop(self):
        self.running = False


class InputHandler:
    """Dispatches client input messages; see module docstring for the vocabulary."""

    def __init__(self, injector: Injector, *, gamepads: Optional[GamepadHub] = None,
                 clipboard: Optional[Clipboard] = None, enable_clipboard: str = "true",
                 enable_binary_clipboard: bool = False,
                 send_clipboard: Optional[Callable[[bytes, str], Awaitable[None]]] = None,
                 layout_offset: Optional[Callable[[str], tuple]] = None,
                 on_client_fps: Optional[Callable[[int], None]] = None,
                 on_client_latency: Optional[Callable[[int], None]] = None,
                 on_set_fps: Optional[Callable[[int], None]] = None,
                 on_resize: Optional[Callable[[bool, Optional[str]], None]] = None,
                 on_client_stats: Optional[Callable[[str, str], None]] = None):
        self.inj = injector
        self.gamepads = gamepads
        self.clipboard = clipboard or Clipboard()
        self.enable_clipboard = enable_clipboard          # "true" | "in" | "out" | "false"
        self.enable_binary_clipboard = enable_binary_clipboard
        self.send_clipboard = send_clipboard
        self.layout_offset = layout_offset or (lambda did: (0, 0))
        self.on_client_fps = on_client_fps or (lambda fps: None)
        self.on_client_latency = on_client_latency or (lambda ms: None)
        self.on_set_fps = on_set_fps or (lambda fps: None)
        self.on_resize = on_resize or (lambda enabled, res: None)
        self.on_client_stats = on_client_stats or (lambda kind, data: None)
        self.button_mask = 0
        self.last_xy = (-1, -1)
        self.modifiers: set[int] = set()
        self.typed_atomically: set[int] = set()
        self.multipart = protocol.ClipboardAssembler()
        self.pointer_visible = True
        self.ping_start: Optional[float] = None
        self.latency_ms = 0.0
        self._clip_task: Optional[asyncio.Task] = None

    # ------------------------------------------------------------------ keyboard
    @property
    def shift(self) -> bool:
        return bool(self.modifiers & SHIFT_KEYSYMS)

    def key(self, keysym: int, down: bool):
        self.inj.key(keysym, down, self.shift)

    async def reset_keyboard(self):
        for ks in RESET_KEYSYMS:
            self.inj.key(ks, False, False)
        self.modifiers.clear()

    def type_text(self, text: str):
        """Types text independent of the current modifier state (``co,end``)."""
        for ch in text:
            ks = char_to_keysym(ch)
            self.inj.key(ks, True, self.shift)
            self.inj.key(ks, False, self.shift)

    def key_down(self, keysym: int):
        if keysym in MODIFIER_KEYSYMS:
            self.modifiers.add(keysym)
        ch = keysym_to_char(keysym)
        # Non-letter printables without a shortcut modifier are typed atomically so
        # a client/server layout mismatch cannot leave stuck or wrong modifiers.
        shortcut_mods = self.modifiers - SHIFT_KEYSYMS
        if ch is not None and not ch.isalpha() and not shortcut_mods:
            self.type_text(ch)
            self.typed_atomically.add(keysym)
            return
        self.key(keysym, True)

    def key_up(self, keysym: int):
        if keysym in MODIFIER_KEYSYMS:
            self.modifiers.discard(keysym)
        if keysym in self.typed_atomically:
            self.typed_atomically.discard(keysym)
            return
        self.key(keysym, False)

    # ------------------------------------------------------------------ pointer
    def mouse(self, x: int, y: int, mask: int, magnitude: int, relative: bool, display_id: str = "primary"):
        if relative:
            if x or y:
                self.inj.motion_rel(x, y)
        else:
            ox, oy = self.layout_offset(display_id)
            fx, fy = x + ox, y + oy
            if (fx, fy) != self.last_xy:
                self.inj.motion(fx, fy)
                self.last_xy = (fx, fy)
        if mask == self.button_mask:
            return
        changed = mask ^ self.button_mask
        for bit in range(8):
            if not changed & (1 << bit):
                continue
            pressed = bool(mask & (1 << bit))
            if bit in (0, 1, 2):
                self.inj.button((BTN_LEFT, BTN_MIDDLE, BTN_RIGHT)[bit], pressed)
            elif bit in (3, 4):
                if magnitude > 0:
                    if pressed:
                        b = WHEEL_DOWN if bit == 3 else WHEEL_UP
                        for _ in range(max(1, magnitude)):
                            self.inj.button(b, True)
                            self.inj.button(b, False)
                elif pressed:  # Back / Forward mouse buttons -> Alt+Left / Alt+Right
                    arrow = XK_LEFT if bit == 3 else XK_RIGHT
                    for ks, down in ((XK_ALT_L, True), (arrow, True), (arrow, False), (XK_ALT_L, False)):
                        self.inj.key(ks, down, False)
            elif bit in (6, 7) and magnitude > 0 and pressed:
                b = WHEEL_LEFT if bit == 6 else WHEEL_RIGHT
                for _ in range(max(1, magnitude)):
                    self.inj.button(b, True)
                    self.inj.button(b, False)
        self.button_mask = mask

    # ------------------------------------------------------------------ clipboard
    def _clip_in(self) -> bool:
        return self.enable_clipboard in ("true", "in")

    def _clip_out(self) -> bool:
        return self.enable_clipboard in ("true", "out")

    async def clipboard_monitor(self, interval: float = 0.5):
        """Polls the X clipboard and pushes changes to clients (outbound sync)."""
        last = None
        while True:
            if self._clip_out() and self.send_clipboard is not None:
                data, mime = await self.clipboard.read(self.enable_binary_clipboard)
                if data is not None:
                    raw = data.encode() if isinstance(data, str) else data
                    if raw != last:
                        last = raw
                        await self.send_clipboard(raw, mime)
            await asyncio.sleep(interval)

    def start_clipboard_monitor(self):
        if self.clipboard.available and (self._clip_task is None or self._clip_task.done()):
            self._clip_task = asyncio.create_task(self.clipboard_monitor())

    async def update_binary_clipboard_setting(self, enabled: bool):
        self.enable_binary_clipboard = bool(enabled)

    # ------------------------------------------------------------------ dispatch
    async def on_message(self, msg: str, display_id: str = "primary"):
        toks = msg.split(",")
        t = toks[0]
        try:
            if t == "kd":
                self.key_down(int(toks[1]))
            elif t == "ku":
                self.key_up(int(toks[1]))
            elif t == "kr":
                await self.reset_keyboard()
            elif t in ("m", "m2"):
                try:
                    x, y, mask, mag = (int(v) for v in toks[1:5])
                    rel = t == "m2"
                except (ValueError, IndexError):
                    x, y, mask, mag, rel = 0, 0, self.button_mask, 0, False
                self.mouse(x, y, mask, mag, rel, display_id)
            elif t == "p":
                self.pointer_visible = bool(int(toks[1]))
            elif t in ("vb", "ab"):
                log.debug("bitrate hint %s=%s (ignored in websocket mode)", t, toks[1])
            elif t == "js":
                await self._gamepad(toks)
            elif t == "cw":
                if self._clip_in():
                    await self.clipboard.write(base64.b64decode(toks[1]).decode("utf-8", "ignore"))
            elif t == "cb":
                if self._clip_in() and self.enable_binary_clipboard:
                    _, mime, b64 = toks
                    await self.clipboard.write(base64.b64decode(b64), mime)
            elif t == "cws":
                if self._clip_in():
                    self.multipart.start("text/plain", int(toks[1]))
            elif t == "cbs":
                if self._clip_in():
                    self.multipart.start(toks[1], int(toks[2]))
            elif t in ("cwd", "cbd"):
                self.multipart.data(toks[1])
            elif t in ("cwe", "cbe"):
                done = self.multipart.end()
                if done is not None:
                    mime, data = done
                    if mime == "text/plain":
                        await self.clipboard.write(data.decode("utf-8", "ignore"))
                    else:
                        await self.clipboard.write(data, mime)
                else:
                    log.warning("multipart clipboard size mismatch; dropped")
            elif t == "cr":
                if self._clip_out() and self.send_clipboard is not None:
                    data, mime = await self.clipboard.read(self.enable_binary_clipboard)
                    if data is not None:
                        await self.send_clipboard(data.encode() if isinstance(data, str) else data, mime)
            elif t == "_arg_fps":
                self.on_set_fps(int(toks[1]))
            elif t == "_arg_resize":
                if len(toks) == 3:
                    enabled, res = toks[1].lower() == "true", toks[2]
                    parsed = None
                    try:
                        w, h = protocol.parse_resolution(res)
                        parsed = f"{w + w % 2}x{h + h % 2}"
                    except ValueError:
                        pass
                    self.on_resize(enabled, parsed)
            elif t == "_f":
                self.on_client_fps(int(toks[1]))
            elif t == "_l":
                self.on_client_latency(int(toks[1]))
            elif t in ("_stats_video", "_stats_audio"):
                self.on_client_stats(t, ",".join(toks[1:]))
            elif t == "co" and len(toks) > 1 and toks[1] == "end":
                self.type_text(msg[len("co,end,"):])
            elif t == "pong":
                if self.ping_start is not None:
                    self.latency_ms = (time.time() - self.ping_start) / 2 * 1000
            else:
                log.info("unknown input message: %s", msg[:100])
        except (ValueError, IndexError) as e:
            log.warning("malformed input message %r: %s", msg[:100], e)

    async def _gamepad(self, toks):
        if self.gamepads is None:
            return
        cmd, slot = toks[1], int(toks[2])
        if cmd == "c":
            try:
                name = base64.b64decode(toks[3]).decode("latin-1", "ignore")[:255]
            except (ValueError, IndexError):
                name = f"ClientGamepad{slot}"
            self.gamepads.connect(slot, name, int(toks[4]), int(toks[5]))
        elif cmd == "d":
            self.gamepads.disconnect(slot)
        elif cmd == "b":
            self.gamepads.button(slot, int(toks[3]), float(toks[4]))
        elif cmd == "a":
            self.gamepads.axis(slot, int(toks[3]), float(toks[4]))

    async def close(self):
        if self._clip_task:
            self._clip_task.cancel()
        if self.gamepads:
            await self.gamepads.close()
        self.inj.close()
