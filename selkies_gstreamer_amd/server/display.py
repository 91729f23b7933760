"""Display geometry: multi-monitor layout, CVT modelines, xrandr, DPI and cursor size.

Behavior parity with the reference (selkies.py:216-418 resize helpers, 442-800
DPI helpers, 2616-2779 reconfigure_displays): the primary client plus at most one
secondary display are laid out side by side (right/left/down/up), the X screen
framebuffer becomes the bounding box (width aligned to 8), one xrandr logical
monitor is created per display, and a capture region is started per display.

Differences by design: the modeline is computed here with the VESA CVT formula
(no ``cvt``/``gtf`` binaries required), and every X tool is optional — without
an X server the layout still drives the capture regions (synthetic source), so
the server runs headless on a GPU node.
"""
from __future__ import annotations

import asyncio
import logging
import math
import os
import re
import shutil
from typing import Optional

log = logging.getLogger("display")

MAX_W, MAX_H = 7680, 4320


# --------------------------------------------------------------------------- layout
def compute_layout(displays: dict) -> tuple[dict, int, int]:
    """displays: {id: {'width', 'height', 'position'}} -> (layouts, total_w, total_h).

    layouts[id] = {'x','y','w','h'}; the total width is aligned up to 8.
    """
    primary = displays.get("primary")
    sec_id = next((d for d in displays if d != "primary"), None)
    layouts: dict = {}
    tw = th = 0
    if primary and not sec_id:
        pw, ph = primary.get("width", 0), primary.get("height", 0)
        if pw > 0 and ph > 0:
            layouts["primary"] = {"x": 0, "y": 0, "w": pw, "h": ph}
            tw, th = pw, ph
    elif primary and sec_id:
        pw, ph = primary.get("width", 0), primary.get("height", 0)
        sec = displays[sec_id]
        sw, sh = sec.get("width", 0), sec.get("height", 0)
        pos = sec.get("position", "right")
        if min(pw, ph, sw, sh) > 0:
            if pos == "left":
                layouts[sec_id] = {"x": 0, "y": 0, "w": sw, "h": sh}
                layouts["primary"] = {"x": sw, "y": 0, "w": pw, "h": ph}
                tw, th = pw + sw, max(ph, sh)
            elif pos == "down":
                layouts["primary"] = {"x": 0, "y": 0, "w": pw, "h": ph}
                layouts[sec_id] = {"x": 0, "y": ph, "w": sw, "h": sh}
                tw, th = max(pw, sw), ph + sh
            elif pos == "up":
                layouts[sec_id] = {"x": 0, "y": 0, "w": sw, "h": sh}
                layouts["primary"] = {"x": 0, "y": sh, "w": pw, "h": ph}
                tw, th = max(pw, sw), ph + sh
            else:  # right (default)
                layouts["primary"] = {"x": 0, "y": 0, "w": pw, "h": ph}
                layouts[sec_id] = {"x": pw, "y": 0, "w": sw, "h": sh}
                tw, th = pw + sw, max(ph, sh)
    if tw:
        tw = (tw + 7) & ~7
    return layouts, tw, th


def fit_resolution(w: int, h: int, max_w: int = MAX_W, max_h: int = MAX_H) -> tuple[int, int]:
    """Scales (w, h) down to fit max_w x max_h keeping the aspect; even dims."""
    if w <= max_w and h <= max_h:
        return w, h
    aspect = w / h
    if w > max_w:
        w, h = max_w, int(max_w / aspect)
    if h > max_h:
        h, w = max_h, int(max_h * aspect)
    return w - w % 2, h - h % 2


# --------------------------------------------------------------------------- CVT
def cvt_modeline(width: int, height: int, refresh: float = 60.0) -> tuple[str, str]:
    """VESA CVT (standard blanking) modeline -> (name, xrandr --newmode params).

    Produces the same timings as the ``cvt`` utility, e.g. 1920x1080@60 ->
    ``173.00 1920 2048 2248 2576 1080 1083 1088 1120 -hsync +vsync``.
    """
    CELL, MIN_VPORCH, MIN_VBPORCH, MIN_VSYNC_BP_US = 8, 3, 6, 550.0
    HSYNC_PCT, C_PRIME, M_PRIME, CLOCK_STEP = 8.0, 30.0, 300.0, 0.25
    hpix = (width // CELL) * CELL
    vlines = height
    aspect = width / height
    vsync = 10
    for ratio, vs in ((4 / 3, 4), (16 / 9, 5), (16 / 10, 6), (5 / 4, 7), (15 / 9, 7)):
        if abs(aspect - ratio) < 0.01:
            vsync = vs
            break
    h_period = (1.0 / refresh - MIN_VSYNC_BP_US / 1e6) / (vlines + MIN_VPORCH) * 1e6
    vsync_bp = math.floor(MIN_VSYNC_BP_US / h_period) + 1
    if vsync_bp < vsync + MIN_VBPORCH:
        vsync_bp = vsync + MIN_VBPORCH
    total_v = vlines + vsync_bp + MIN_VPORCH
    duty = C_PRIME - M_PRIME * h_period / 1000.0
    duty = max(duty, 20.0)
    hblank = math.floor(hpix * duty / (100.0 - duty) / (2 * CELL)) * (2 * CELL)
    total_h = hpix + hblank
    clock = math.floor(total_h / h_period / CLOCK_STEP) * CLOCK_STEP
    hsync = math.floor(HSYNC_PCT / 100.0 * total_h / CELL) * CELL
    hsync_end = hpix + hblank // 2
    hsync_start = hsync_end - hsync
    vsync_start = vlines + MIN_VPORCH
    vsync_end = vsync_start + vsync
    real_refresh = clock * 1e6 / (total_h * total_v)
    name = f"{width}x{height}_{real_refresh:.2f}"
    params = (f"{clock:.2f} {hpix} {hsync_start} {hsync_end} {total_h} "
              f"{vlines} {vsync_start} {vsync_end} {total_v} -hsync +vsync")
    return name, params


# --------------------------------------------------------------------------- xrandr
def display_env(display: Optional[str], base: Optional[dict] = None) -> Optional[dict]:
    """Environment for an X tool aimed at ``display``; None keeps the process's own.

    A session host serves several desktops from one process (parallel/multi.py),
    so the X display is passed to every subprocess explicitly instead of being
    read from the process-wide DISPLAY."""
    if not display:
        return base
    env = dict(os.environ if base is None else base)
    env["DISPLAY"] = display
    return env


async def run(cmd: list[str], env: Optional[dict] = None, timeout: float = 10.0) -> tuple[int, str]:
    """Runs a command; (returncode, stdout). Missing binaries -> (127, '')."""
    if shutil.which(cmd[0]) is None:
        return 127, ""
    try:
        p = await asyncio.create_subprocess_exec(*cmd, stdout=asyncio.subprocess.PIPE,
                                                 stderr=asyncio.subprocess.STDOUT, env=env)
        out, _ = await asyncio.wait_for(p.communicate(), timeout)
        return p.returncode, out.decode("utf-8", "replace")
    except (OSError, asyncio.TimeoutError) as e:
        log.warning("%s failed: %s", cmd[0], e)
        return 1, ""


_SCREEN = re.compile(r"^(\S+) connected")
_CURRENT = re.compile(r".*current (\d+)\s*x\s*(\d+)")
_MODE = re.compile(r"^\s+(\d+x\d+)\s+\d+\.\d+")


def parse_xrandr(text: str) -> tuple[Optional[str], Optional[str], list[str]]:
    """xrandr output -> (screen name, current 'WxH', modes of that screen)."""
    screen = current = None
    modes: list[str] = []
    in_screen = False
    for line in text.splitlines():
        m = _CURRENT.match(line)
        if m and current is None:
            current = f"{m.group(1)}x{m.group(2)}"
        m = _SCREEN.match(line)
        if m:
            if screen is None:
                screen = m.group(1)
            in_screen = m.group(1) == screen
            continue
        if in_screen:
            m = _MODE.match(line)
            if m:
                modes.append(m.group(1))
            elif line and not line[0].isspace():
                in_screen = False
    return screen, current, sorted(set(modes))


class XrandrDisplay:
    """Applies a layout to the X screen with xrandr (no-op without X)."""

    def __init__(self, display: Optional[str] = None):
        self.display = display if display is not None else os.environ.get("DISPLAY")
        self.env = display_env(self.display)
        self.available = bool(self.display) and shutil.which("xrandr") is not None

    async def _x(self, *args):
        return await run(["xrandr", *args], env=self.env)

    async def query(self):
        if not self.available:
            return None, None, []
        rc, out = await self._x()
        if rc != 0:
            return None, None, []
        return parse_xrandr(out)

    async def monitors(self) -> list[str]:
        rc, out = await self._x("--listmonitors")
        if rc != 0:
            return []
        names = []
        for line in out.splitlines()[1:]:
            parts = line.split()
            if len(parts) >= 4:
                names.append(parts[1].lstrip("+*"))
        return names

    async def ensure_mode(self, screen: str, mode: str, modes: list[str]) -> bool:
        if mode in modes:
            return True
        w, h = (int(x) for x in mode.split("x"))
        _, params = cvt_modeline(w, h)
        rc, _ = await self._x("--newmode", mode, *params.split())
        rc2, _ = await self._x("--addmode", screen, mode)
        if rc2 != 0:
            await self._x("--delmode", screen, mode)
            await self._x("--rmmode", mode)
            return False
        return True

    async def apply(self, layouts: dict, total_w: int, total_h: int) -> bool:
        screen, _, modes = await self.query()
        if not screen:
            return False
        for name in await self.monitors():
            if name.startswith("selkies-"):
                await self._x("--delmonitor", name)
        mode = f"{total_w}x{total_h}"
        if not await self.ensure_mode(screen, mode, modes):
            log.error("cannot create mode %s", mode)
            return False
        await self._x("--fb", mode, "--output", screen, "--mode", mode)
        for did, l in layouts.items():
            geom = f"{l['w']}/0x{l['h']}/0+{l['x']}+{l['y']}"
            await self._x("--setmonitor", f"selkies-{did}", geom, screen)
        if "primary" in layouts:
            await self._x("--output", screen, "--primary")
        return True

    async def clear(self):
        if not self.available:
            return
        for name in await self.monitors():
            if name.startswith("selkies-"):
                await self._x("--delmonitor", name)


# --------------------------------------------------------------------------- DPI
def detect_desktop(which=shutil.which) -> str:
    """Desktop session, in the reference's probe order (selkies.py:704-741):
    KDE -> XFCE -> MATE -> i3 -> Openbox -> generic."""
    for name, probes in (("kde", ("startplasma-x11",)), ("xfce", ("xfce4-session",)), ("mate", ("mate-session",)),
                         ("i3", ("i3",)), ("openbox", ("openbox-session", "openbox"))):
        if any(which(p) for p in probes):
            return name
    return "generic"


def merge_setting_file(path: str, key: str, line: str, sep: str = " ") -> None:
    """Sets one key of a `key<sep>value` style file, keeping every other line.

    The reference rewrites ~/.Xresources and ~/.xsettingsd wholesale (selkies.py:442-480),
    losing the user's other resources; this keeps them and only replaces `key`."""
    try:
        with open(path) as f:
            lines = f.read().splitlines()
    except OSError:
        lines = []
    out, done = [], False
    for ln in lines:
        k = ln.split(sep, 1)[0].strip().rstrip(":")
        if k == key.rstrip(":"):
            if not done:
                out.append(line)
                done = True
            continue
        out.append(ln)
    if not done:
        out.append(line)
    tmp = path + ".selkies-tmp"
    with open(tmp, "w") as f:
        f.write("\n".join(out) + "\n")
    os.replace(tmp, path)


async def _xrdb_dpi(dpi: int, display: Optional[str] = None) -> bool:
    """Xft.dpi through xrdb -merge (the resource database, not a file rewrite) plus
    the Xft/DPI key of ~/.xsettingsd with a SIGHUP to a running xsettingsd."""
    if not shutil.which("xrdb"):
        return False
    ok = False
    try:
        p = await asyncio.create_subprocess_exec("xrdb", "-merge", stdin=asyncio.subprocess.PIPE,
                                                 stdout=asyncio.subprocess.DEVNULL, stderr=asyncio.subprocess.PIPE,
                                                 env=display_env(display))
        await p.communicate(f"Xft.dpi: {dpi}\n".encode())
        ok = p.returncode == 0
        merge_setting_file(os.path.expanduser("~/.Xresources"), "Xft.dpi:", f"Xft.dpi:   {dpi}", sep=":")
        merge_setting_file(os.path.expanduser("~/.xsettingsd"), "Xft/DPI", f"Xft/DPI {dpi * 1024}")
        rc, out = await run(["pgrep", "-x", "xsettingsd"])
        if rc == 0 and out.strip():
            await run(["kill", "-HUP", out.split()[0]])
    except OSError as e:
        log.warning("xrdb DPI update failed: %s", e)
    return ok


async def _xfconf_dpi(dpi: int, display: Optional[str] = None) -> bool:
    if not shutil.which("xfconf-query"):
        return False
    env = display_env(display, await _session_env("xfce4-session"))
    rc, _ = await run(["xfconf-query", "-c", "xsettings", "-p", "/Xft/DPI", "-s", str(dpi), "--create", "-t", "int"],
                      env=env)
    return rc == 0


async def _mate_dpi(dpi: int, display: Optional[str] = None) -> bool:
    if not shutil.which("gsettings"):
        return False
    scale = dpi / 96.0
    factor = int(scale) if scale == int(scale) else 1
    env = display_env(display)
    rc, _ = await run(["gsettings", "set", "org.mate.interface", "window-scaling-factor", str(max(1, factor))], env=env)
    rc2, _ = await run(["gsettings", "set", "org.mate.font-rendering", "dpi", str(dpi)], env=env)
    return rc == 0 or rc2 == 0


async def set_dpi(dpi: int, desktop: Optional[str] = None, display: Optional[str] = None) -> bool:
    """Applies DPI the way the running desktop takes it: XFCE through xfconf only
    (xrdb as well would scale twice), MATE through gsettings + xrdb, KDE / i3 /
    Openbox / anything else through xrdb."""
    try:
        dpi = int(dpi)
    except (TypeError, ValueError):
        return False
    if dpi <= 0:
        return False
    de = desktop or detect_desktop()
    if de == "xfce":
        ok = await _xfconf_dpi(dpi, display)
    elif de == "mate":
        ok = await _mate_dpi(dpi, display)
        ok = await _xrdb_dpi(dpi, display) or ok
    else:
        ok = await _xrdb_dpi(dpi, display)
    if not ok:
        log.warning("no DPI method succeeded for %d (desktop %s)", dpi, de)
    return ok


class WindowManagerSwap:
    """Multi-monitor: XFCE's and KDE's window managers place windows on the X
    screen, not on the per-display xrandr monitors, so with more than one display
    the session switches to openbox with a minimal config (selkies.py:2631-2647).
    Unlike the reference this also switches back when the session returns to one
    display."""

    def __init__(self, which=shutil.which, runner=None, display: Optional[str] = None):
        self.which = which
        self.env = display_env(display)
        self.desktop = detect_desktop(which)
        self.supported = self.desktop in ("xfce", "kde") and which("openbox") is not None
        self.swapped = False
        self._runner = runner

    @staticmethod
    async def _spawn(cmd, env=None):
        try:
            await asyncio.create_subprocess_exec(*cmd, stdout=asyncio.subprocess.DEVNULL, env=env,
                                                 stderr=asyncio.subprocess.DEVNULL, start_new_session=True)
        except OSError as e:
            log.warning("%s failed: %s", cmd[0], e)

    async def update(self, display_count: int) -> None:
        if not self.supported:
            return
        if display_count > 1 and not self.swapped:
            cfg = os.path.join(os.environ.get("XDG_RUNTIME_DIR") or "/tmp", "selkies_openbox.xml")
            try:
                with open(cfg, "w") as f:
                    f.write("<openbox_config></openbox_config>\n")
                cmd = ["openbox", "--config-file", cfg, "--replace"]
            except OSError:
                cmd = ["openbox", "--replace"]
            await self._call(cmd)
            self.swapped = True
        elif display_count <= 1 and self.swapped:
            native = ["xfwm4", "--replace"] if self.desktop == "xfce" else ["kwin_x11", "--replace"]
            await self._call(native)
            self.swapped = False

    async def _call(self, cmd):
        if self._runner is None:
            await self._spawn(cmd, self.env)
        else:
            await self._runner(cmd)


async def set_cursor_size(size: int, display: Optional[str] = None) -> bool:
    ok = False
    if shutil.which("xfconf-query"):
        env = display_env(display, await _session_env("xfce4-session"))
        rc, _ = await run(["xfconf-query", "-c", "xsettings", "-p", "/Gtk/CursorThemeSize", "-s", str(size),
                           "--create", "-t", "int"], env=env)
        ok |= rc == 0
    if shutil.which("gsettings"):
        rc, _ = await run(["gsettings", "set", "org.mate.peripherals-mouse", "cursor-size", str(size)],
                          env=display_env(display))
        ok |= rc == 0
    return ok


async def _session_env(proc_name: str) -> Optional[dict]:
    rc, out = await run(["pgrep", "-o", "-x", proc_name])
    if rc != 0 or not out.strip():
        return None
    try:
        with open(f"/proc/{out.split()[0]}/environ", "rb") as f:
            items = f.read().split(b"\0")
    except OSError:
        return None
    env = dict(kv.decode(errors="replace").split("=", 1) for kv in items if b"=" in kv)
    return env if "DBUS_SESSION_BUS_ADDRESS" in env else None
