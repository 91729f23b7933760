"""Builds the native library (C++ runtime + gfx950 HIP kernels) in-tree.

`python -m selkies_gstreamer_amd.ops.build` compiles every ``csrc/**/*.cpp`` and
``csrc/**/*.hip`` with ``hipcc --offload-arch=gfx950`` into
``selkies_gstreamer_amd/_lib/libselkies_native.so`` (incremental by mtime).
The .so travels with the repository snapshot to the GPU box (gpurun).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CSRC = ROOT / "csrc"
_STAMPS = bool(os.environ.get("SK_STAMPS_BUILD"))
BUILD = ROOT / "build" / ("native_stamps" if _STAMPS else "native")
LIBDIR = ROOT / "selkies_gstreamer_amd" / "_lib"
# diagnostic build with s_memtime stamps (SK_STAMPS_BUILD=1) goes to its own library
LIB = LIBDIR / ("libselkies_native_stamps.so" if _STAMPS else "libselkies_native.so")
ARCH = os.environ.get("SK_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CXXFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
    "-Wno-unused-variable", "-Wno-unused-but-set-variable", "-Wno-unused-lambda-capture",
    f"-I{CSRC}", f"-I{CSRC / 'codec'}", f"-I{CSRC / 'runtime'}",
] + (["-DSK_STAMPS", f"-DSK_STAMP_BLOCK={int(os.environ.get('SK_STAMP_BLOCK', '0'))}",
       f"-DSK_STAMP_STEP0={int(os.environ.get('SK_STAMP_STEP0', '0'))}"]
      if os.environ.get("SK_STAMPS_BUILD") else [])


RTC_LIB = LIBDIR / "libselkies_rtc.so"


def _sources():
    # csrc/rtc is host-only (OpenSSL) and goes into its own library, see build_rtc()
    return sorted([p for p in CSRC.rglob("*") if p.suffix in (".cpp", ".hip") and "rtc" not in p.parts])


def _headers_mtime() -> float:
    return max((p.stat().st_mtime for p in CSRC.rglob("*.h")), default=0.0)


def _compile(src: Path, hdr_mtime: float, verbose: bool) -> Path:
    obj = BUILD / (str(src.relative_to(CSRC)).replace("/", "__") + ".o")
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr_mtime):
        return obj
    cmd = [HIPCC, *CXXFLAGS, "-c", str(src), "-o", str(obj)]
    if src.suffix == ".hip":
        cmd[1:1] = ["-x", "hip"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip() and verbose:
        print(r.stderr, file=sys.stderr)
    return obj


def build(verbose: bool = False, jobs: int | None = None) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    hdr = _headers_mtime()
    srcs = _sources()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, verbose), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if not LIB.exists() or LIB.stat().st_mtime < newest:
        # RUNPATH: the library's own dependencies (HIP runtime, the system libstdc++) resolve
        # without the RPATH of a host executable that ships an older libstdc++
        # (gst-launch-1.0 from /opt/conda loading libgsthip)
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(LIB), *map(str, objs),
               "-lpthread", "-ldl", "-Wl,--enable-new-dtags,-rpath,/opt/rocm/lib:/usr/lib/x86_64-linux-gnu"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
    return LIB


def build_rtc(verbose: bool = False) -> Path:
    """WebRTC transport core (DTLS-SRTP, SRTP, RTP packetisation): plain C++ on OpenSSL."""
    LIBDIR.mkdir(parents=True, exist_ok=True)
    srcs = sorted((CSRC / "rtc").glob("*.cpp"))
    newest = max(p.stat().st_mtime for p in [*srcs, *(CSRC / "rtc").glob("*.h")])
    if RTC_LIB.exists() and RTC_LIB.stat().st_mtime >= newest:
        return RTC_LIB
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-deprecated-declarations", *map(str, srcs), "-o", str(RTC_LIB), "-lssl", "-lcrypto"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"rtc build failed\n{r.stdout}\n{r.stderr}")
    return RTC_LIB


def main(argv=None) -> int:
    """``selkies-build``: the HIP engine library, the WebRTC media library and the shims."""
    argv = sys.argv[1:] if argv is None else argv
    print(build(verbose="-v" in argv))
    print(build_rtc(verbose="-v" in argv))
    from .build_shims import build_shims
    print(build_shims())
    return 0


if __name__ == "__main__":
    sys.exit(main())
