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
