"""Builds the GStreamer plugin ``libgsthip.so`` (csrc/gst/gsthip.c) in-tree.

The elements (hiph264enc, hiph265enc, hipav1enc, hipconvert) link against the
GStreamer found through its pkg-config files - by default the GStreamer 1.14 under
``/opt/conda`` (``SK_GST_PREFIX`` overrides) - and against libselkies_native.so.
The image has no ``pkg-config`` binary, so the ``.pc`` files are read here
(variables, Cflags, Libs, Requires resolved recursively).

Output: ``selkies_gstreamer_amd/_lib/gstreamer-1.0/libgsthip.so`` (RUNPATH
``$ORIGIN/..`` for libselkies_native.so). Use it with
``GST_PLUGIN_PATH=<that dir>`` (see :func:`gst_env`).
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
SRC = ROOT / "csrc" / "gst" / "gsthip.c"
SRCS = sorted((ROOT / "csrc" / "gst").glob("*.c"))
LIBDIR = ROOT / "selkies_gstreamer_amd" / "_lib"
PLUGDIR = LIBDIR / "gstreamer-1.0"
PLUGIN = PLUGDIR / "libgsthip.so"
PREFIX = Path(os.environ.get("SK_GST_PREFIX", "/opt/conda"))


def _pc_path(name: str) -> Path | None:
    for d in (PREFIX / "lib" / "pkgconfig", PREFIX / "share" / "pkgconfig"):
        p = d / f"{name}.pc"
        if p.exists():
            return p
    return None


def _pc_read(name: str) -> dict:
    p = _pc_path(name)
    if p is None:
        raise FileNotFoundError(f"{name}.pc not found under {PREFIX}")
    var: dict[str, str] = {}
    fields: dict[str, str] = {}
    for line in p.read_text().splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        m = re.match(r"^([A-Za-z0-9_.]+)\s*=\s*(.*)$", line)
        if m and ":" not in m.group(1):
            var[m.group(1)] = m.group(2)
            continue
        m = re.match(r"^([A-Za-z.]+)\s*:\s*(.*)$", line)
        if m:
            fields[m.group(1)] = m.group(2)

    def expand(s: str) -> str:
        for _ in range(10):
            s2 = re.sub(r"\$\{([^}]+)\}", lambda mm: var.get(mm.group(1), ""), s)
            if s2 == s:
                break
            s = s2
        return s
    return {k: expand(v) for k, v in fields.items()}


def pkg_flags(*names: str) -> tuple[list[str], list[str]]:
    """(cflags, libs) of the packages and everything they Require, like pkg-config."""
    cflags: list[str] = []
    libs: list[str] = []
    seen: set[str] = set()

    def visit(n: str) -> None:
        if n in seen:
            return
        seen.add(n)
        f = _pc_read(n)
        for r in re.split(r"[,\s]+", f.get("Requires", "")):
            r = r.strip()
            if r and not re.match(r"^[<>=0-9.]+$", r):
                visit(r)
        for t in f.get("Cflags", "").split():
            if t not in cflags:
                cflags.append(t)
        for t in f.get("Libs", "").split():
            if t not in libs:
                libs.append(t)
    for n in names:
        visit(n)
    return cflags, libs


def available() -> bool:
    """GStreamer headers / .pc files and the launcher are present."""
    return _pc_path("gstreamer-video-1.0") is not None and (PREFIX / "bin" / "gst-launch-1.0").exists()


def gst_env(base: dict | None = None) -> dict:
    """Environment for gst-launch / gst-inspect that finds libgsthip (and the prefix's plugins)."""
    env = dict(os.environ if base is None else base)
    paths = [str(PLUGDIR), str(PREFIX / "lib" / "gstreamer-1.0")]
    env["GST_PLUGIN_PATH"] = os.pathsep.join(paths)
    env["GST_PLUGIN_SYSTEM_PATH"] = str(PREFIX / "lib" / "gstreamer-1.0")
    # a registry of our own, so no stale cache from another build is used
    env["GST_REGISTRY"] = str(PLUGDIR / f"registry.{os.uname().machine}.bin")
    scanner = PREFIX / "libexec" / "gstreamer-1.0" / "gst-plugin-scanner"
    if scanner.exists():
        env["GST_PLUGIN_SCANNER"] = str(scanner)
    return env


def gst_bin(tool: str) -> str:
    return str(PREFIX / "bin" / tool)


def build(verbose: bool = False) -> Path:
    if not available():
        raise FileNotFoundError(f"no GStreamer development files under {PREFIX}")
    from selkies_gstreamer_amd.ops.build import build as build_native
    native = build_native()
    PLUGDIR.mkdir(parents=True, exist_ok=True)
    newest = max([p.stat().st_mtime for p in SRCS + sorted((ROOT / "csrc" / "gst").glob("*.h"))] +
                 [native.stat().st_mtime, Path(__file__).stat().st_mtime])
    if PLUGIN.exists() and PLUGIN.stat().st_mtime >= newest:
        return PLUGIN
    cflags, libs = pkg_flags("gstreamer-video-1.0", "gstreamer-base-1.0")
    cc = shutil.which("gcc") or "cc"
    cmd = [cc, "-O2", "-fPIC", "-shared", "-Wall", "-Wno-unused-function", "-std=gnu11", *cflags, *map(str, SRCS),
           "-o", str(PLUGIN), *libs, f"-L{LIBDIR}", "-lselkies_native",
           f"-Wl,--enable-new-dtags,-rpath,$ORIGIN/..:{PREFIX / 'lib'}", "-Wl,--no-undefined"]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"libgsthip build failed\n{r.stdout}\n{r.stderr}")
    reg = PLUGDIR / f"registry.{os.uname().machine}.bin"
    if reg.exists():
        reg.unlink()
    return PLUGIN


if __name__ == "__main__":
    print(build(verbose=True))
