"""ABI tests of the LD_PRELOAD shims (csrc/shims): a real child process with the
joystick interposer preloaded opens /dev/input/js0 and /dev/input/event1000,
queries them with ioctls and receives events from the gamepad socket server;
the fake libudev is enumerated through ctypes like SDL does."""
import ctypes
import fcntl
import json
import os
import struct
import subprocess
import sys

import pytest

from selkies_gstreamer_amd.ops.build_shims import build_shims

CHILD = r'''
import fcntl, json, os, struct, sys
def IOC(d, t, nr, size): return (d << 30) | (size << 16) | (ord(t) << 8) | nr
R = 2
js = os.open("/dev/input/js0", os.O_RDONLY)
ev = os.open("/dev/input/event1000", os.O_RDONLY)
out = {}
out["axes"] = fcntl.ioctl(js, IOC(R, "j", 0x11, 1), b"\0")[0]
out["buttons"] = fcntl.ioctl(js, IOC(R, "j", 0x12, 1), b"\0")[0]
out["version"] = struct.unpack("I", fcntl.ioctl(js, IOC(R, "j", 0x01, 4), b"\0" * 4))[0]
out["name"] = fcntl.ioctl(js, IOC(R, "j", 0x13, 128), b"\0" * 128).split(b"\0")[0].decode()
btnmap = struct.unpack("11H", fcntl.ioctl(js, IOC(R, "j", 0x34, 22), b"\0" * 22))
out["btnmap0"] = btnmap[0]
bus, ven, prod, ver = struct.unpack("4H", fcntl.ioctl(ev, IOC(R, "E", 0x02, 8), b"\0" * 8))
out["id"] = [bus, ven, prod, ver]
out["evname"] = fcntl.ioctl(ev, IOC(R, "E", 0x06, 64), b"\0" * 64).split(b"\0")[0].decode()
keybits = fcntl.ioctl(ev, IOC(R, "E", 0x20 + 1, 96), b"\0" * 96)
out["has_btn_a"] = bool(keybits[0x130 // 8] & (1 << (0x130 % 8)))
absz = struct.unpack("6i", fcntl.ioctl(ev, IOC(R, "E", 0x40 + 2, 24), b"\0" * 24))
out["absz"] = [absz[1], absz[2]]
out["access"] = os.access("/dev/input/js1", os.R_OK)
print(json.dumps(out), flush=True)
e = os.read(js, 8)
out2 = {"js": list(struct.unpack("<IhBB", e))[1:]}
d = b""
while len(d) < 48:
    d += os.read(ev, 48 - len(d))
out2["ev"] = list(struct.unpack_from("<qqHHi", d, 0))[2:]
print(json.dumps(out2), flush=True)
'''


@pytest.fixture(scope="module")
def shims():
    return build_shims()


SERVER = r'''
import asyncio, sys
from selkies_gstreamer_amd.server.gamepad import GamepadHub

async def main(sock_dir):
    hub = GamepadHub(sock_dir, slots=4)
    await hub.start()
    print("ready", flush=True)
    loop = asyncio.get_running_loop()
    while True:
        line = await loop.run_in_executor(None, sys.stdin.readline)
        if not line or line.strip() == "quit":
            break
        slot, idx, val = line.split()
        hub.button(int(slot), int(idx), float(val))
    await hub.close()

asyncio.run(main(sys.argv[1]))
'''


def test_js_interposer_end_to_end(shims, tmp_path):
    """Gamepad socket server and LD_PRELOADed client run as two real processes."""
    interposer, _ = shims
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    srv = subprocess.Popen([sys.executable, "-c", SERVER, str(tmp_path)], cwd=root, stdin=subprocess.PIPE,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           env=dict(os.environ, PYTHONPATH=root))
    p = None
    try:
        assert srv.stdout.readline().strip() == "ready", srv.stderr.read()
        env = dict(os.environ, LD_PRELOAD=str(interposer), SELKIES_INTERPOSER_SOCKET_DIR=str(tmp_path))
        p = subprocess.Popen([sys.executable, "-c", CHILD], env=env, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, text=True)
        line = p.stdout.readline()
        assert line, p.stderr.read()
        info = json.loads(line)
        assert info["axes"] == 8 and info["buttons"] == 11
        assert info["version"] == 0x020100
        assert info["name"] == info["evname"] == "Microsoft X-Box 360 pad"
        assert info["btnmap0"] == 0x130
        assert info["id"] == [0x03, 0x045E, 0x028E, 0x0114]
        assert info["has_btn_a"] and info["absz"] == [0, 255] and info["access"] is True
        srv.stdin.write("0 0 1.0\n")                 # A pressed on pad 0
        srv.stdin.flush()
        line2 = p.stdout.readline()
        assert line2, p.stderr.read()
        ev = json.loads(line2)
        assert ev["js"] == [1, 1, 0]                  # value 1, JS_EVENT_BUTTON, button 0
        assert ev["ev"] == [1, 0x130, 1]              # EV_KEY BTN_A 1
        assert p.wait(10) == 0
    finally:
        for proc in (p, srv):
            if proc is not None and proc.poll() is None:
                proc.kill()
                proc.wait(5)


def test_interposer_passthrough(shims, tmp_path):
    """Non-device paths and fds are untouched by the preloaded interposer."""
    interposer, _ = shims
    f = tmp_path / "x.txt"
    f.write_text("hello")
    code = f"import os; fd = os.open({str(f)!r}, os.O_RDONLY); print(os.read(fd, 5).decode()); os.close(fd)"
    env = dict(os.environ, LD_PRELOAD=str(interposer), SELKIES_INTERPOSER_SOCKET_DIR=str(tmp_path))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=30)
    assert out.stdout.strip() == "hello", out.stderr
    code = "import os, errno\ntry:\n    os.open('/dev/input/js2', os.O_RDONLY)\nexcept OSError as e:\n    print(e.errno)"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=30)
    assert out.stdout.strip() == str(2)  # ENOENT when no server socket is listening


def test_fake_udev_enumeration(shims):
    _, udev_path = shims
    L = ctypes.CDLL(str(udev_path))
    vp, cp = ctypes.c_void_p, ctypes.c_char_p
    for name, res, args in [
        ("udev_new", vp, []), ("udev_enumerate_new", vp, [vp]), ("udev_enumerate_add_match_subsystem", ctypes.c_int, [vp, cp]),
        ("udev_enumerate_add_match_property", ctypes.c_int, [vp, cp, cp]), ("udev_enumerate_scan_devices", ctypes.c_int, [vp]),
        ("udev_enumerate_get_list_entry", vp, [vp]), ("udev_list_entry_get_next", vp, [vp]),
        ("udev_list_entry_get_name", cp, [vp]), ("udev_device_new_from_syspath", vp, [vp, cp]),
        ("udev_device_get_devnode", cp, [vp]), ("udev_device_get_property_value", cp, [vp, cp]),
        ("udev_device_get_parent_with_subsystem_devtype", vp, [vp, cp, cp]),
        ("udev_device_get_sysattr_value", cp, [vp, cp]), ("udev_device_unref", vp, [vp]),
        ("udev_enumerate_unref", vp, [vp]), ("udev_unref", vp, [vp]), ("udev_monitor_new_from_netlink", vp, [vp, cp]),
        ("udev_monitor_get_fd", ctypes.c_int, [vp]), ("udev_monitor_receive_device", vp, [vp]),
        ("udev_monitor_unref", vp, [vp]), ("udev_device_new_from_devnum", vp, [vp, ctypes.c_char, ctypes.c_ulong])]:
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    u = L.udev_new()
    e = L.udev_enumerate_new(u)
    L.udev_enumerate_add_match_subsystem(e, b"input")
    L.udev_enumerate_add_match_property(e, b"ID_INPUT_JOYSTICK", b"1")
    assert L.udev_enumerate_scan_devices(e) == 0
    nodes, vendors = set(), set()
    it = L.udev_enumerate_get_list_entry(e)
    count = 0
    while it:
        d = L.udev_device_new_from_syspath(u, L.udev_list_entry_get_name(it))
        assert d
        node = L.udev_device_get_devnode(d)
        if node:
            nodes.add(node.decode())
            assert L.udev_device_get_property_value(d, b"ID_VENDOR_ID") == b"045e"
            usb = L.udev_device_get_parent_with_subsystem_devtype(d, b"usb", b"usb_device")
            vendors.add(L.udev_device_get_sysattr_value(usb, b"idVendor"))
        L.udev_device_unref(d)
        count += 1
        it = L.udev_list_entry_get_next(it)
    assert count == 12
    assert nodes == {f"/dev/input/js{i}" for i in range(4)} | {f"/dev/input/event{1000 + i}" for i in range(4)}
    assert vendors == {b"045e"}
    d = L.udev_device_new_from_devnum(u, b"c", os.makedev(13, 64 + 1002))
    assert L.udev_device_get_devnode(d) == b"/dev/input/event1002"
    m = L.udev_monitor_new_from_netlink(u, b"udev")
    assert L.udev_monitor_get_fd(m) >= 0 and not L.udev_monitor_receive_device(m)
    L.udev_monitor_unref(m)
    L.udev_enumerate_unref(e)
    L.udev_unref(u)
    syms = subprocess.run(["objdump", "-T", str(udev_path)], capture_output=True, text=True).stdout
    for ver in ("LIBUDEV_183", "LIBUDEV_189", "LIBUDEV_196", "LIBUDEV_199", "LIBUDEV_215", "LIBUDEV_247"):
        assert ver in syms


REF_UDEV_SYM = "/root/reference/addons/fake-udev/libudev.sym"


def test_fake_udev_exports_every_reference_symbol(shims):
    _, udev_path = shims
    """Every symbol of the reference's version script (libudev.sym) is exported, with its
    version node; a game linked against any of them resolves under the preload."""
    import re
    if not os.path.exists(REF_UDEV_SYM):
        pytest.skip("reference tree not mounted")
    want = {}
    node = None
    for line in open(REF_UDEV_SYM):
        m = re.match(r"\s*(LIBUDEV_\d+)\s*\{", line)
        if m:
            node = m.group(1)
            continue
        m = re.match(r"\s*(udev_\w+)\s*;", line)
        if m and node:
            want[m.group(1)] = node
    assert len(want) >= 90
    out = subprocess.run(["objdump", "-T", str(udev_path)], capture_output=True, text=True).stdout
    have = {}
    for line in out.splitlines():
        f = line.split()
        if len(f) >= 2 and f[-1].startswith("udev_"):
            have[f[-1]] = f[-2]
    missing = sorted(set(want) - set(have))
    assert not missing, missing
    wrong = {k: (have[k], v) for k, v in want.items() if have[k].strip("()") != v}
    assert not wrong, wrong


def test_fake_udev_children_devicenode_sysnum(shims):
    _, udev_path = shims
    """udev_enumerate_scan_children lists the parent and what is below it;
    add_match_devicenode / add_match_sysnum filter like libudev (glob patterns)."""
    L = ctypes.CDLL(str(udev_path))
    L.udev_new.restype = ctypes.c_void_p
    L.udev_enumerate_new.restype = ctypes.c_void_p
    L.udev_enumerate_new.argtypes = [ctypes.c_void_p]
    L.udev_enumerate_get_list_entry.restype = ctypes.c_void_p
    L.udev_enumerate_get_list_entry.argtypes = [ctypes.c_void_p]
    L.udev_list_entry_get_next.restype = ctypes.c_void_p
    L.udev_list_entry_get_next.argtypes = [ctypes.c_void_p]
    L.udev_list_entry_get_name.restype = ctypes.c_char_p
    L.udev_list_entry_get_name.argtypes = [ctypes.c_void_p]
    for f in ("udev_enumerate_add_match_devicenode", "udev_enumerate_add_match_sysnum",
              "udev_enumerate_add_match_subsystem"):
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    L.udev_enumerate_add_match_parent.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for f in ("udev_enumerate_scan_devices", "udev_enumerate_scan_children", "udev_enumerate_unref"):
        getattr(L, f).argtypes = [ctypes.c_void_p]
    L.udev_device_new_from_syspath.restype = ctypes.c_void_p
    L.udev_device_new_from_syspath.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    L.udev_device_get_parent_with_subsystem_devtype.restype = ctypes.c_void_p
    L.udev_device_get_parent_with_subsystem_devtype.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
    L.udev_device_get_syspath.restype = ctypes.c_char_p
    L.udev_device_get_syspath.argtypes = [ctypes.c_void_p]

    def names(e):
        out, it = [], L.udev_enumerate_get_list_entry(e)
        while it:
            out.append(L.udev_list_entry_get_name(it).decode())
            it = L.udev_list_entry_get_next(it)
        return out
    u = L.udev_new()
    e = L.udev_enumerate_new(u)
    L.udev_enumerate_add_match_devicenode(e, b"/dev/input/js*")
    assert L.udev_enumerate_scan_devices(e) == 0
    js = names(e)
    assert len(js) == 4 and all(p.split("/")[-1].startswith("js") for p in js)
    L.udev_enumerate_unref(e)
    e = L.udev_enumerate_new(u)
    L.udev_enumerate_add_match_subsystem(e, b"input")
    L.udev_enumerate_add_match_sysnum(e, b"1002")
    assert L.udev_enumerate_scan_devices(e) == 0
    assert [p.split("/")[-1] for p in names(e)] == ["event1002"]
    L.udev_enumerate_unref(e)
    # children of pad 1's USB device: its input node and the js / event nodes below it
    d = L.udev_device_new_from_syspath(u, js[1].encode())
    usb = L.udev_device_get_parent_with_subsystem_devtype(d, b"usb", b"usb_device")
    assert usb
    e = L.udev_enumerate_new(u)
    assert L.udev_enumerate_scan_children(e) < 0          # no parent set
    L.udev_enumerate_add_match_parent(e, usb)
    assert L.udev_enumerate_scan_children(e) == 0
    kids = names(e)
    assert L.udev_device_get_syspath(usb).decode() in kids and js[1] in kids
    assert not any(k in kids for k in js if k != js[1])
    L.udev_enumerate_unref(e)

