"""Builds the CPU-side LD_PRELOAD shims in-tree (csrc/shims):

* ``_lib/libselkies_js_interposer.so`` — virtual /dev/input/js0-3 + event1000-1003
  backed by the gamepad sockets (reference addons/js-interposer, same socket ABI);
* ``_lib/udev/libudev.so.1`` — fake libudev describing the same four pads
  (reference addons/fake-udev), exported with libudev's symbol versions.

Usage in a session: ``LD_PRELOAD=<_lib>/libselkies_js_interposer.so:<_lib>/udev/libudev.so.1 <game>``.
"""
from __future__ import annotations

import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
SHIMS = ROOT / "csrc" / "shims"
OUT = Path(__file__).resolve().parents[1] / "_lib"

CFLAGS = ["-O2", "-fPIC", "-shared", "-Wall", "-Wextra", "-Wno-unused-parameter", "-std=gnu11"]


def _run(cmd):
    subprocess.run(cmd, check=True)


def _stale(out: Path, *srcs: Path) -> bool:
    return not out.exists() or any(s.stat().st_mtime > out.stat().st_mtime for s in srcs)


def build_shims(cc: str = "gcc") -> list[Path]:
    OUT.mkdir(parents=True, exist_ok=True)
    (OUT / "udev").mkdir(exist_ok=True)
    js = OUT / "libselkies_js_interposer.so"
    src = SHIMS / "js_interposer.c"
    if _stale(js, src):
        _run([cc, *CFLAGS, "-o", str(js), str(src), "-ldl", "-lpthread"])
    udev = OUT / "udev" / "libudev.so.1"
    usrc, umap = SHIMS / "fake_udev.c", SHIMS / "libudev.map"
    if _stale(udev, usrc, umap):
        _run([cc, *CFLAGS, "-fvisibility=hidden", "-Wl,-soname,libudev.so.1", f"-Wl,--version-script={umap}",
              "-o", str(udev), str(usrc)])
    return [js, udev]


if __name__ == "__main__":
    for p in build_shims():
        print(p)
