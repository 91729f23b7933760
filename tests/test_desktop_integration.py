"""Desktop integration without a desktop: DPI per desktop environment (reference
selkies.py:704-741), config files updated without clobbering, the multi-monitor
window-manager swap (selkies.py:2631-2647) and the non-blocking microphone sink."""
import asyncio
import threading
import time

from selkies_gstreamer_amd.server import audio, display, protocol


def _which(*present):
    return lambda name: f"/usr/bin/{name}" if name in present else None


def test_detect_desktop_order():
    assert display.detect_desktop(_which("startplasma-x11", "xfce4-session")) == "kde"
    assert display.detect_desktop(_which("xfce4-session", "openbox")) == "xfce"
    assert display.detect_desktop(_which("mate-session")) == "mate"
    assert display.detect_desktop(_which("i3")) == "i3"
    assert display.detect_desktop(_which("openbox")) == "openbox"
    assert display.detect_desktop(_which()) == "generic"


def test_merge_setting_file_keeps_other_lines(tmp_path):
    xr = tmp_path / ".Xresources"
    xr.write_text("XTerm*faceName: Mono\nXft.dpi: 96\nURxvt.scrollBar: false\n")
    display.merge_setting_file(str(xr), "Xft.dpi:", "Xft.dpi:   144", sep=":")
    assert xr.read_text().splitlines() == ["XTerm*faceName: Mono", "Xft.dpi:   144", "URxvt.scrollBar: false"]
    xs = tmp_path / ".xsettingsd"
    display.merge_setting_file(str(xs), "Xft/DPI", "Xft/DPI 98304")   # created when missing
    display.merge_setting_file(str(xs), "Net/ThemeName", 'Net/ThemeName "Adwaita"')
    display.merge_setting_file(str(xs), "Xft/DPI", "Xft/DPI 147456")
    assert xs.read_text().splitlines() == ["Xft/DPI 147456", 'Net/ThemeName "Adwaita"']


def test_set_dpi_dispatch(monkeypatch):
    calls = []

    async def fake(name, ok=True):
        calls.append(name)
        return ok
    monkeypatch.setattr(display, "_xfconf_dpi", lambda d, disp=None: fake("xfconf"))
    monkeypatch.setattr(display, "_mate_dpi", lambda d, disp=None: fake("mate"))
    monkeypatch.setattr(display, "_xrdb_dpi", lambda d, disp=None: fake("xrdb"))
    for de, exp in (("xfce", ["xfconf"]), ("mate", ["mate", "xrdb"]), ("kde", ["xrdb"]), ("i3", ["xrdb"]),
                    ("generic", ["xrdb"])):
        calls.clear()
        assert asyncio.run(display.set_dpi(120, desktop=de))
        assert calls == exp, de
    assert not asyncio.run(display.set_dpi(0, desktop="kde"))
    assert not asyncio.run(display.set_dpi("x", desktop="kde"))


def test_wm_swap_round_trip():
    ran = []

    async def runner(cmd):
        ran.append(cmd[0])
    wm = display.WindowManagerSwap(which=_which("xfce4-session", "openbox"), runner=runner)
    assert wm.supported

    async def go():
        await wm.update(1)
        await wm.update(2)
        await wm.update(3)   # already swapped
        await wm.update(1)
    asyncio.run(go())
    assert ran == ["openbox", "xfwm4"] and not wm.swapped
    assert not display.WindowManagerSwap(which=_which("i3", "openbox"), runner=runner).supported


def test_mic_sink_push_does_not_block():
    sink = audio.MicSink()
    release = threading.Event()
    written = []

    def slow_write(stream, chunk):   # PulseAudio's buffer is full: the write blocks
        release.wait(5)
        written.append(len(chunk))
        return True
    sink._write = slow_write
    sink.ready = True
    chunk = b"\x01\x00" * 480                        # 20 ms
    t = time.perf_counter()
    for _ in range(300):                             # 6 s of audio while the writer is stuck
        assert sink.push(chunk) == len(chunk)
    assert time.perf_counter() - t < 0.5             # never waited on the writer
    assert len(sink.buffer) <= protocol.MIC_BUFFER_MAX and sink.dropped > 0
    release.set()
    deadline = time.time() + 5
    while sink.buffer and time.time() < deadline:
        time.sleep(0.01)
    assert not sink.buffer and sum(written) > 0
    sink.close()
    assert sink._thread is None


def test_mic_sink_close_never_frees_under_a_blocked_write():
    """close() waits 2 s; a writer still inside pa_simple_write then owns the stream
    and frees it itself when the write returns. A reopened sink gets a live writer."""
    freed = []

    class PA:
        def pa_simple_free(self, s):
            freed.append(s)
    sink = audio.MicSink()
    sink.pa = PA()
    release = threading.Event()
    entered = threading.Event()

    def blocked_write(stream, chunk):
        entered.set()
        release.wait(10)
        return True
    sink._write = blocked_write
    sink.stream, sink.ready = "s1", True
    sink.push(b"\x00\x00" * 480)
    assert entered.wait(5)
    t = time.perf_counter()
    sink.close()
    assert 1.5 < time.perf_counter() - t < 5 and freed == []     # not freed under the write
    release.set()
    deadline = time.time() + 5
    while not freed and time.time() < deadline:
        time.sleep(0.01)
    assert freed == ["s1"]                                         # the writer freed it afterwards
    got = []
    sink._write = lambda stream, chunk: got.append(stream) or True
    sink.stream, sink.ready = "s2", True
    sink.push(b"\x00\x00" * 480)
    deadline = time.time() + 5
    while not got and time.time() < deadline:
        time.sleep(0.01)
    assert got == ["s2"]                                           # reopened sink writes again
    sink.close()
    assert freed == ["s1", "s2"]
