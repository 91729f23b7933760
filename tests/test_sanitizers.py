"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer.

The CPU reference encoders (H.264 with the stripe controller and deblocking,
JPEG) and the G.711/G.722 codecs are compiled with g++
-fsanitize=address,undefined and driven by tests/native/sanitize_harness.cpp;
any report fails the test (halt_on_error). GPU code is exercised by the gpu tier
(GPU ASan is not available on this pool).
"""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "csrc"
GXX = shutil.which("g++")

pytestmark = pytest.mark.skipif(GXX is None, reason="g++ not installed")


def test_cpu_encoders_and_codecs_clean_under_asan_ubsan(tmp_path):
    srcs = [CSRC / "codec" / n for n in ("h264_cpu.cpp", "h264_control.cpp", "jpeg_cpu.cpp", "telephony.cpp")]
    srcs.append(ROOT / "tests" / "native" / "sanitize_harness.cpp")
    exe = tmp_path / "harness"
    cmd = [GXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", f"-I{CSRC}", f"-I{CSRC / 'codec'}", f"-I{CSRC / 'runtime'}",
           *map(str, srcs), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
    assert "sanitized run ok" in r.stdout
