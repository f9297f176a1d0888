"""NUMA-local placement policy (docs/DESIGN_HISTORY.md §6, libhdfs3_amd/csrc/numa.cpp) checked on fake sysfs
trees: a device's PCI function -> its NUMA node (bus/pci/devices/<bdf>/numa_node) -> that node's
CPUs (devices/system/node/node<N>/cpulist). The worker, receiver and loader threads of a device bind
to those CPUs (intersected with the process's allowed CPUs) before they pin their staging."""
import ctypes
import os

import pytest


def fake_sysfs(root, bdf, node, cpulist):
    d = os.path.join(root, "bus", "pci", "devices", bdf)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "numa_node"), "w") as f:
        f.write(f"{node}\n")
    if cpulist is not None and node >= 0:
        n = os.path.join(root, "devices", "system", "node", f"node{node}")
        os.makedirs(n, exist_ok=True)
        with open(os.path.join(n, "cpulist"), "w") as f:
            f.write(cpulist + "\n")


def cpus(root, bdf, cap=1024):
    from libhdfs3_amd import _native

    out = (ctypes.c_int * cap)()
    n = _native.lib().hdfs3_numa_cpus(root.encode(), bdf.encode(), out, cap)
    return n if n <= 0 else list(out[:min(n, cap)])


def test_two_socket_node(tmp_path):
    root = str(tmp_path)
    fake_sysfs(root, "0000:05:00.0", 0, "0-31,64-95")
    fake_sysfs(root, "0000:85:00.0", 1, "32-63,96-127")
    assert cpus(root, "0000:05:00.0") == list(range(0, 32)) + list(range(64, 96))
    assert cpus(root, "0000:85:00.0") == list(range(32, 64)) + list(range(96, 128))
    # hipDeviceGetPCIBusId may report upper-case hex: sysfs names are lower case
    fake_sysfs(root, "0000:c5:00.0", 1, "32-63,96-127")
    assert cpus(root, "0000:C5:00.0") == list(range(32, 64)) + list(range(96, 128))


def test_unknown_node_leaves_threads_alone(tmp_path):
    root = str(tmp_path)
    fake_sysfs(root, "0000:05:00.0", -1, None)
    assert cpus(root, "0000:05:00.0") == 0       # numa_node -1: no binding
    assert cpus(root, "0000:99:00.0") == 0       # no such device in the tree


def test_single_cpus_and_malformed_lists(tmp_path):
    root = str(tmp_path)
    fake_sysfs(root, "0000:01:00.0", 3, "7")
    assert cpus(root, "0000:01:00.0") == [7]
    fake_sysfs(root, "0000:02:00.0", 4, "1-")
    assert cpus(root, "0000:02:00.0") < 0        # -EINVAL: not a cpulist
    fake_sysfs(root, "0000:03:00.0", 5, "")
    assert cpus(root, "0000:03:00.0") < 0


def test_count_beyond_buffer(tmp_path):
    root = str(tmp_path)
    fake_sysfs(root, "0000:05:00.0", 0, "0-255")
    assert cpus(root, "0000:05:00.0", cap=4) == [0, 1, 2, 3]
    from libhdfs3_amd import _native

    assert _native.lib().hdfs3_numa_cpus(root.encode(), b"0000:05:00.0", None, 0) == 256
