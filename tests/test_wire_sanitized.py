"""CPU: the wire codec that parses datanode bytes (csrc/client/wire.cpp) under AddressSanitizer
and UndefinedBehaviorSanitizer (host code only), driven by tests/native/wire_fuzz.cpp:
encode->decode identities, hostile/mutated inputs into every decoder, and the PacketHeader
sanity rules of PacketHeader.cpp:72-86."""
import os
import shutil
import subprocess

import pytest

from util import REPO

SRC = os.path.join(REPO, "tests", "native", "wire_fuzz.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_wire_codec_under_asan_ubsan(tmp_path):
    exe = tmp_path / "wire_fuzz"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I", os.path.join(REPO, "libhdfs3_amd", "csrc"), SRC,
           os.path.join(REPO, "libhdfs3_amd", "csrc", "client", "wire.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True)
    # verify_asan_link_order=0: the environment may preload other libraries ahead of ASan
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([str(exe), "60000"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "wire fuzz ok" in out.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_net_reads_under_asan_ubsan(tmp_path):
    """csrc/client/net.cpp's socket reads (round 5: recv what is buffered first, one MSG_WAITALL recv
    under SO_RCVTIMEO for a large remainder, and read_fully2's scatter read of a packet's checksums and
    data) against a writer sending random-sized pieces with pauses: every byte in place, timeouts and EOF
    reported as -ETIMEDOUT / -ECONNRESET."""
    exe = tmp_path / "net_reads"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I", os.path.join(REPO, "libhdfs3_amd", "csrc"), os.path.join(REPO, "tests", "native", "net_reads.cpp"),
           os.path.join(REPO, "libhdfs3_amd", "csrc", "client", "net.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert "net reads ok" in out.stdout
