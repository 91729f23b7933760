"""NUMA binding helpers (parallel/numa.py) on a fake sysfs tree."""
import os

from selkies_gstreamer_amd.parallel import numa


def test_parse_cpulist():
    assert numa.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa.parse_cpulist("") == set()


def test_node_lookup(tmp_path):
    dev = tmp_path / "bus/pci/devices/0000:c1:00.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text("1\n")
    node = tmp_path / "devices/system/node/node1"
    node.mkdir(parents=True)
    (node / "cpulist").write_text("4-7\n")
    assert numa.numa_node_of_pci("0000:c1:00.0", str(tmp_path)) == 1
    assert numa.node_cpus(1, str(tmp_path)) == {4, 5, 6, 7}
    (dev / "numa_node").write_text("-1\n")
    assert numa.numa_node_of_pci("0000:c1:00.0", str(tmp_path)) is None
    assert numa.numa_node_of_pci("0000:00:00.0", str(tmp_path)) is None


def test_bind_without_gpu_is_a_noop():
    before = os.sched_getaffinity(0)
    assert numa.bind_to_gpu(0) is None          # no HIP device in this container
    assert os.sched_getaffinity(0) == before
