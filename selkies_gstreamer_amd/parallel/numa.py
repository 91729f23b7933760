"""NUMA placement of a GPU's host-side work.

Every frame crosses PCIe from pinned host memory (profiles/r1_host_bounds_and_tracing.md:
one GPU ingests ~53 GB/s); on a multi-socket node a process whose pinned frames
sit on the far socket pays the inter-socket link on every upload, and with eight
GPUs streaming at once that link saturates. Each rank / session process binds
itself to the CPUs of the NUMA node its GPU hangs off *before* allocating pinned
buffers, so first-touch places them locally (bench.py, parallel/launcher.py).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional


def parse_cpulist(text: str) -> set[int]:
    out: set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def gpu_pci_address(device: int) -> Optional[str]:
    from ..ops.native import lib
    buf = ctypes.create_string_buffer(64)
    L = lib()
    L.sk_hip_pci_bus_id.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    if L.sk_hip_pci_bus_id(device, buf, 64) != 0:
        return None
    return buf.value.decode().lower()


def numa_node_of_pci(addr: str, sysfs: str = "/sys") -> Optional[int]:
    try:
        with open(os.path.join(sysfs, "bus/pci/devices", addr, "numa_node")) as f:
            n = int(f.read().strip())
        return n if n >= 0 else None
    except (OSError, ValueError):
        return None


def node_cpus(node: int, sysfs: str = "/sys") -> set[int]:
    try:
        with open(os.path.join(sysfs, f"devices/system/node/node{node}/cpulist")) as f:
            return parse_cpulist(f.read())
    except OSError:
        return set()


def bind_to_gpu(device: int, sysfs: str = "/sys") -> Optional[int]:
    """Restricts this process to the CPUs of the GPU's NUMA node (intersected with
    the CPUs it may use). Returns the node, or None when nothing was changed."""
    if os.environ.get("SK_NUMA_BIND", "1") == "0":
        return None
    addr = gpu_pci_address(device)
    node = numa_node_of_pci(addr, sysfs) if addr else None
    if node is None:
        return None
    cpus = node_cpus(node, sysfs) & os.sched_getaffinity(0)
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return node
