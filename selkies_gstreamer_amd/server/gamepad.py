"""Virtual gamepads served to the joystick interposer (csrc/shims/js_interposer.c).

Socket ABI (shared with the reference's interposer, input_handler.py:46-760 and
addons/js-interposer/joystick_interposer.c:320-330, so either side can be mixed):

* per slot i in 0..3 two unix sockets: ``<dir>/selkies_js{i}.sock`` (joystick
  API) and ``<dir>/selkies_event{1000+i}.sock`` (evdev);
* on connect the server writes one ``js_config_t`` (1360 bytes: name[255], pad,
  vendor, product, version, num_btns, num_axes (u16), btn_map[512] (u16),
  axes_map[64] (u8), 6 pad bytes); the interposer answers with one byte =
  ``sizeof(long)`` of the game process (4 or 8);
* then the server streams ``struct js_event`` (8 B: u32 ms, s16 value, u8 type,
  u8 number) or ``struct input_event`` + ``SYN_REPORT`` (2 x 16/24 B depending on
  the client's ``long``).

Browser "standard gamepad" indices are mapped onto an Xbox 360 pad: buttons to
BTN_*, LT/RT buttons to the Z/RZ axes, the d-pad to HAT0X/HAT0Y.
"""
from __future__ import annotations

import asyncio
import ctypes
import logging
import os
import struct
import time
from dataclasses import dataclass
from typing import Optional

log = logging.getLogger("gamepad")

NAME_LEN, MAX_BTNS, MAX_AXES = 255, 512, 64
JS_CONFIG_SIZE = 1360
JS_EVENT_BUTTON, JS_EVENT_AXIS = 0x01, 0x02
EV_SYN, EV_KEY, EV_ABS = 0x00, 0x01, 0x03

BTN_A, BTN_B, BTN_X, BTN_Y = 0x130, 0x131, 0x133, 0x134
BTN_TL, BTN_TR, BTN_SELECT, BTN_START, BTN_MODE = 0x136, 0x137, 0x13A, 0x13B, 0x13C
BTN_THUMBL, BTN_THUMBR = 0x13D, 0x13E
ABS_X, ABS_Y, ABS_Z, ABS_RX, ABS_RY, ABS_RZ, ABS_HAT0X, ABS_HAT0Y = 0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x10, 0x11

AXIS_MIN, AXIS_MAX = -32767, 32767
NUM_SLOTS = 4


class JsConfig(ctypes.Structure):
    """Byte-exact mirror of the interposer's ``js_config_t``."""
    _fields_ = [
        ("name", ctypes.c_char * NAME_LEN),
        ("vendor", ctypes.c_uint16),
        ("product", ctypes.c_uint16),
        ("version", ctypes.c_uint16),
        ("num_btns", ctypes.c_uint16),
        ("num_axes", ctypes.c_uint16),
        ("btn_map", ctypes.c_uint16 * MAX_BTNS),
        ("axes_map", ctypes.c_uint8 * MAX_AXES),
        ("final_alignment_padding", ctypes.c_uint8 * 6),
    ]


assert ctypes.sizeof(JsConfig) == JS_CONFIG_SIZE


@dataclass(frozen=True)
class PadModel:
    name: str
    vendor: int
    product: int
    version: int
    buttons: tuple          # internal button index -> BTN_* code
    axes: tuple             # internal axis index -> ABS_* code
    client_btn: dict        # browser button -> internal button index
    client_axis: dict       # browser axis -> internal axis index
    btn_to_axis: dict       # browser button -> internal axis (analog triggers)
    dpad: dict              # browser button -> (internal hat axis, direction)
    trigger_axes: frozenset
    hat_axes: frozenset


XPAD = PadModel(
    name="Microsoft X-Box 360 pad", vendor=0x045E, product=0x028E, version=0x0114,
    buttons=(BTN_A, BTN_B, BTN_X, BTN_Y, BTN_TL, BTN_TR, BTN_SELECT, BTN_START, BTN_MODE, BTN_THUMBL, BTN_THUMBR),
    axes=(ABS_X, ABS_Y, ABS_Z, ABS_RX, ABS_RY, ABS_RZ, ABS_HAT0X, ABS_HAT0Y),
    client_btn={0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 8: 6, 9: 7, 10: 9, 11: 10, 16: 8},
    client_axis={0: 0, 1: 1, 2: 3, 3: 4},
    btn_to_axis={6: 2, 7: 5},
    dpad={12: (7, -1), 13: (7, 1), 14: (6, -1), 15: (6, 1)},
    trigger_axes=frozenset({2, 5}), hat_axes=frozenset({6, 7}),
)


def pack_js_config(model: PadModel = XPAD) -> bytes:
    c = JsConfig()
    name = model.name.encode("utf-8")[:NAME_LEN - 1]
    c.name = name
    c.vendor, c.product, c.version = model.vendor, model.product, model.version
    c.num_btns, c.num_axes = len(model.buttons), len(model.axes)
    for i, code in enumerate(model.buttons[:MAX_BTNS]):
        c.btn_map[i] = code
    for i, code in enumerate(model.axes[:MAX_AXES]):
        c.axes_map[i] = code
    return bytes(c)


def unpack_js_config(data: bytes) -> JsConfig:
    if len(data) != JS_CONFIG_SIZE:
        raise ValueError("js_config_t must be 1360 bytes")
    return JsConfig.from_buffer_copy(data)


def _axis_value(v: float, trigger: bool, hat: bool, js: bool) -> int:
    if hat:
        h = int(max(-1, min(1, round(v))))
        return h * AXIS_MAX if js else h
    if trigger:  # 0..1: full axis range on the joystick API, 0..255 on evdev (xpad's ABS_Z/ABS_RZ)
        return int(AXIS_MIN + v * (AXIS_MAX - AXIS_MIN)) if js else int(round(max(0.0, min(1.0, v)) * 255))
    return int(AXIS_MIN + (v + 1.0) / 2.0 * (AXIS_MAX - AXIS_MIN))  # -1..1


@dataclass
class PadEvent:
    js_type: int
    js_number: int
    js_value: int
    ev_type: int
    ev_code: int
    ev_value: int


def map_event(model: PadModel, index: int, value: float, is_button: bool) -> Optional[PadEvent]:
    """Browser gamepad event -> (js_event, input_event) pair, or None if unmapped."""
    trigger = hat = False
    if is_button:
        if index in model.dpad:
            axis, direction = model.dpad[index]
            hat, v = True, direction * int(value)
            kind = EV_ABS
            internal = axis
        elif index in model.btn_to_axis:
            internal = model.btn_to_axis[index]
            trigger = internal in model.trigger_axes
            kind, v = EV_ABS, value
        else:
            internal = model.client_btn.get(index)
            kind, v = EV_KEY, int(value)
    else:
        internal = model.client_axis.get(index)
        if internal is None:
            return None
        trigger, hat = internal in model.trigger_axes, internal in model.hat_axes
        kind, v = EV_ABS, value
    if internal is None:
        return None
    if kind == EV_KEY:
        if not 0 <= internal < len(model.buttons):
            return None
        iv = int(v)
        return PadEvent(JS_EVENT_BUTTON, internal, iv, EV_KEY, model.buttons[internal], iv)
    if not 0 <= internal < len(model.axes):
        return None
    return PadEvent(JS_EVENT_AXIS, internal, _axis_value(v, trigger, hat, True), EV_ABS, model.axes[internal],
                    _axis_value(v, trigger, hat, False))


def pack_js_event(e: PadEvent, now: Optional[float] = None) -> bytes:
    ms = int((time.time() if now is None else now) * 1000) & 0xFFFFFFFF
    return struct.pack("<IhBB", ms, max(-32768, min(32767, e.js_value)), e.js_type, e.js_number)


def pack_input_events(e: PadEvent, long_size: int, now: Optional[float] = None) -> bytes:
    t = time.time() if now is None else now
    sec = int(t)
    usec = int((t - sec) * 1e6)
    tv = "qq" if long_size == 8 else "ii"
    fmt = f"<{tv}HHi"
    return struct.pack(fmt, sec, usec, e.ev_type, e.ev_code, e.ev_value) + struct.pack(fmt, sec, usec, EV_SYN, 0, 0)


class VirtualGamepad:
    """One slot: serves the js and evdev sockets and fans events out to them."""

    def __init__(self, slot: int, socket_dir: str = "/tmp", model: PadModel = XPAD):
        self.slot, self.model = slot, model
        self.js_path = os.path.join(socket_dir, f"selkies_js{slot}.sock")
        self.ev_path = os.path.join(socket_dir, f"selkies_event{1000 + slot}.sock")
        self.config = pack_js_config(model)
        self.js_clients: dict = {}
        self.ev_clients: dict = {}
        self.servers: list = []
        self.client_name: Optional[str] = None

    async def start(self):
        for path, evdev in ((self.js_path, False), (self.ev_path, True)):
            try:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                if os.path.exists(path):
                    os.unlink(path)
                srv = await asyncio.start_unix_server(lambda r, w, e=evdev: self._client(r, w, e), path=path)
                self.servers.append(srv)
            except OSError as ex:
                log.error("gamepad %d: cannot serve %s: %s", self.slot, path, ex)

    async def _client(self, reader, writer, evdev: bool):
        clients = self.ev_clients if evdev else self.js_clients
        try:
            writer.write(self.config)
            await writer.drain()
            arch = await asyncio.wait_for(reader.readexactly(1), timeout=10.0)
            clients[writer] = arch[0]
            await reader.read()  # returns at EOF (interposer closed the device)
        except (asyncio.IncompleteReadError, asyncio.TimeoutError, ConnectionError):
            pass
        finally:
            clients.pop(writer, None)
            writer.close()

    def emit(self, index: int, value: float, is_button: bool) -> Optional[PadEvent]:
        e = map_event(self.model, index, value, is_button)
        if e is None:
            return None
        if self.js_clients:
            data = pack_js_event(e)
            for w in list(self.js_clients):
                if not w.is_closing():
                    w.write(data)
        for w, long_size in list(self.ev_clients.items()):
            if not w.is_closing():
                w.write(pack_input_events(e, long_size))
        return e

    async def close(self):
        for s in self.servers:
            s.close()
            await s.wait_closed()
        for w in list(self.js_clients) + list(self.ev_clients):
            w.close()
        self.servers = []
        for p in (self.js_path, self.ev_path):
            try:
                os.unlink(p)
            except OSError:
                pass


class GamepadHub:
    """The four persistent pads; browser controllers are associated per slot."""

    def __init__(self, socket_dir: str = "/tmp", slots: int = NUM_SLOTS):
        self.pads = [VirtualGamepad(i, socket_dir) for i in range(slots)]

    async def start(self):
        for p in self.pads:
            await p.start()

    def connect(self, slot: int, name: str, num_axes: int, num_btns: int):
        if 0 <= slot < len(self.pads):
            self.pads[slot].client_name = name
            log.info("gamepad slot %d <- '%s' (%d buttons, %d axes)", slot, name, num_btns, num_axes)

    def disconnect(self, slot: Optional[int] = None):
        for p in self.pads if slot is None else self.pads[slot:slot + 1]:
            p.client_name = None

    def button(self, slot: int, index: int, value: float):
        if 0 <= slot < len(self.pads):
            self.pads[slot].emit(index, value, True)

    def axis(self, slot: int, index: int, value: float):
        if 0 <= slot < len(self.pads):
            self.pads[slot].emit(index, value, False)

    async def close(self):
        for p in self.pads:
            await p.close()
