"""The drop-in boundary as a C++ caller sees it: tests/native/abi_consumer.cpp includes only
include/hdfs3_crc.h, links libhdfs3_crc.so (built by `make`, no Python or torch in the
process) and runs the reference call-site shapes — RemoteBlockReader::verifyChecksum,
LocalBlockReader::readAndVerify, OutputStreamImpl compute, a wire-layout packet arena with
odd offsets, device-resident blocks — checked word for word against the oracle."""
import os
import subprocess

import pytest

from util import REPO

BIN = os.path.join(REPO, "tests", "native", "abi_consumer")


def _run(*args):
    if not os.path.exists(BIN):
        pytest.fail("tests/native/abi_consumer not built (run `make`)")
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=120)


def test_cpp_consumer_refuses_without_device():
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible; the -m gpu test runs the consumer")
    r = _run("nodevice")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "nodevice ok" in r.stdout


@pytest.mark.gpu
def test_cpp_consumer_on_gpu():
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_consumer ok" in r.stdout


CLIENT_BIN = os.path.join(REPO, "tests", "native", "client_consumer")


@pytest.mark.gpu
def test_cpp_client_consumer_round_trip_on_gpu():
    """tests/native/client_consumer.cpp: hdfs3_output_* writes FillBuffer data in 1 KiB
    packets (GPU CRCs checked against the oracle packet by packet), loopback datanodes serve
    the blocks with those words, hdfs3_input_* reads them back (CheckBuffer in 20 KiB + 1
    reads, pread across a block boundary, one failover off a corrupt replica, EOVERFLOW past
    EOF, EIO when every replica is bad)."""
    if not os.path.exists(CLIENT_BIN):
        pytest.fail("tests/native/client_consumer not built (run `make`)")
    r = subprocess.run([CLIENT_BIN], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "client_consumer ok" in r.stdout


HDFS_BIN = os.path.join(REPO, "tests", "native", "hdfs_consumer")


def _hdfs_consumer(*args, timeout=110):
    if not os.path.exists(HDFS_BIN):
        pytest.fail("tests/native/hdfs_consumer not built (run `make`)")
    r = subprocess.run([HDFS_BIN, *args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, r.stdout
    import json
    return json.loads(line[-1])


@pytest.mark.gpu
def test_c_consumer_on_hdfs_h_surface():
    """tests/native/hdfs_consumer.c, plain C against include/hdfs3_hdfs.h (the reference's
    hdfs.h prototypes): hdfsOpenFile/hdfsWrite/hdfsFlush/hdfsSync/hdfsCloseFile with 1 KiB
    packets (GPU words checked against the oracle), then hdfsRead (20 KiB + 1 reads,
    CheckBuffer), hdfsPread across a block boundary, hdfsSeek/hdfsTell/hdfsAvailable, one
    failover off a corrupt replica, EIO when only the corrupt replica is left, and the errno
    of each misuse (ENOTSUP, ENOENT, EINVAL, EOVERFLOW)."""
    j = _hdfs_consumer()
    assert j["hdfs_consumer"] == "ok" and j["blocks"] == 4 and j["bytes"] == 3 * (1 << 20) + 234


@pytest.mark.gpu
def test_config5_1gib_file_through_hdfsRead():
    """BASELINE.json configs[4] at its stated size: a 1 GiB file of 8 x 128 MiB blocks written
    through hdfsWrite (64 KiB packets, every packet's words checked against the oracle), served
    over loopback TCP by two replicas (block 1 of the first corrupt), read back through
    hdfsRead in 4 MiB calls: every byte CheckBuffer'd, one failover, then EIO from the corrupt
    replica alone. Prints the end-to-end rates (docs/DESIGN_HISTORY.md §5.1)."""
    j = _hdfs_consumer("128", "8", timeout=115)
    assert j["hdfs_consumer"] == "ok" and j["blocks"] == 8 and j["bytes"] == 1 << 30
    print(j)
