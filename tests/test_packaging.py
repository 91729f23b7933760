"""Installable package: pyproject console scripts resolve, and the reference's
``selkies`` import names (src/selkies/*) map onto this build's modules."""
import importlib
import subprocess
import sys
from pathlib import Path

import pytest

try:
    import tomllib
except ImportError:   # python 3.10
    import tomli as tomllib

ROOT = Path(__file__).resolve().parents[1]


def test_console_scripts_resolve():
    meta = tomllib.loads((ROOT / "pyproject.toml").read_text())
    scripts = meta["project"]["scripts"]
    assert scripts["selkies"] == "selkies.__main__:main"   # reference pyproject.toml:58-59
    for name, target in scripts.items():
        mod, fn = target.split(":")
        assert callable(getattr(importlib.import_module(mod), fn)), name


@pytest.mark.parametrize("alias,real", [
    ("selkies.settings", "selkies_gstreamer_amd.server.settings"),
    ("selkies.input_handler", "selkies_gstreamer_amd.server.input"),
    ("selkies.legacy.gstwebrtc_app", "selkies_gstreamer_amd.legacy.webrtc_app"),
    ("selkies.webrtc.sdp", "selkies_gstreamer_amd.webrtc.sdp"),
])
def test_reference_import_names(alias, real):
    assert importlib.import_module(alias) is importlib.import_module(real)


def test_selkies_help_runs():
    r = subprocess.run([sys.executable, "-m", "selkies", "--help"], cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "--port" in r.stdout


def test_no_tracked_binaries():
    out = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True).stdout.split()
    elf = [f for f in out if (ROOT / f).is_file() and (ROOT / f).read_bytes()[:4] == b"\x7fELF"]
    assert not elf, elf
