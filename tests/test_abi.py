"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every symbol
include/hdfs3_crc.h declares, and fails loudly (no silent CPU fallback) without a GPU.
No compute calls are made here."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from util import REPO, read_checksum1, read_checksum2

HEADER = os.path.join(REPO, "include", "hdfs3_crc.h")
CLIENT_HEADER = os.path.join(REPO, "include", "hdfs3_client.h")


def declared_functions(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hdfs3_\w+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for must in ["hdfs3_crc_ctx_create", "hdfs3_crc32c_verify", "hdfs3_crc32c_compute",
                 "hdfs3_crc32c_verify_dev", "hdfs3_crc32c_verify_packets", "hdfs3_crc_last_error"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    from libhdfs3_amd import _native

    lib = _native.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding covers exactly the header
    assert sorted(_native.PUBLIC_API) == declared_functions()
    client = declared_functions(CLIENT_HEADER)
    assert client and not [n for n in client if not hasattr(lib, n)]
    assert sorted(_native.CLIENT_API) == client


HDFS_HEADER = os.path.join(REPO, "include", "hdfs3_hdfs.h")


def test_hdfs_h_surface_exported():
    """include/hdfs3_hdfs.h: the hdfs.h functions (reference prototypes) and the namenode
    stand-in are exported by the product library and bound by _native.HDFS_API."""
    from libhdfs3_amd import _native

    src = re.sub(r"/\*.*?\*/", "", open(HDFS_HEADER).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(hdfs[A-Z]\w+|hdfs3_fs_\w+)\s*\(", src)))
    for must in ["hdfsRead", "hdfsPread", "hdfsWrite", "hdfsFlush", "hdfsHFlush", "hdfsSync", "hdfsCloseFile",
                 "hdfsOpenFile", "hdfsGetLastError"]:
        assert must in names
    lib = _native.load()
    assert not [n for n in names if not hasattr(lib, n)]
    assert sorted(_native.HDFS_API) == names


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_product_library_exports_only_the_c_api():
    """No A/B knob, diagnostic or wrong-on-purpose kernel is reachable from libhdfs3_crc.so:
    the variant knob (hdfs3x_set_variant) and every hdfs3x_* hook live only in the measurement
    library libhdfs3_crc_lab.so, and no internal C++ symbol is exported."""
    from libhdfs3_amd import _native

    prod = {s for s in _exported(_native.LIB_PATH) if not s.startswith("__")}
    assert not [s for s in prod if s.startswith("hdfs3x_")]
    assert not [s for s in prod if s.startswith("_Z")]
    assert all(s.startswith("hdfs3_") or re.match(r"hdfs[A-Z]", s) for s in prod), sorted(prod)
    lab = _exported(_native.LAB_PATH)
    assert {"hdfs3x_set_variant", "hdfs3x_stream_read"} <= lab


def test_library_is_gfx950_code_object():
    from libhdfs3_amd import _native

    blob = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_abi_version_and_errors_without_device():
    from libhdfs3_amd import _native

    lib = _native.load()
    assert lib.hdfs3_crc_abi_version() == 1
    p = ctypes.c_void_p()
    # invalid arguments are rejected before any device work
    assert lib.hdfs3_crc32c_verify(None, None, 0, 512, None, 0, None) == -22  # -EINVAL
    assert lib.hdfs3_crc32c_compute(None, None, 16, 0, None) == -22
    if os.environ.get("HIP_VISIBLE_DEVICES", None) == "" or not os.path.exists("/dev/kfd"):
        rc = lib.hdfs3_crc_ctx_create(0, ctypes.byref(p))
        assert rc < 0 and p.value is None
        assert lib.hdfs3_crc_last_error()


def test_engine_refuses_without_gpu_instead_of_falling_back():
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible; covered by -m gpu tests")
    from libhdfs3_amd._native import Hdfs3CrcError
    from libhdfs3_amd.engine import CrcContext

    with pytest.raises(Hdfs3CrcError):
        CrcContext(0)


def test_streaming_host_shim_matches_reference_fixtures():
    # hdfs3_crc32c_update_host = Checksum::update on a raw state (sub-chunk pieces only)
    from libhdfs3_amd.engine import update_host

    for want, s in read_checksum1():
        assert (~update_host(0xFFFFFFFF, s)) & 0xFFFFFFFF == want
    result, lines = read_checksum2()
    st = 0xFFFFFFFF
    for s in lines:
        st = update_host(st, s)
    assert (~st) & 0xFFFFFFFF == result


def test_missing_library_raises(tmp_path):
    from libhdfs3_amd import _native

    with pytest.raises(ImportError):
        _native.load(str(tmp_path / "nope.so"))


@pytest.mark.parametrize("value,want_mib,warns", [("64M", 64, False), ("2G", 2048, False), ("1048576", 1, False),
                                                   ("1.5G", 1024, True), ("64MiB", 1024, True), ("-1", 1024, True),
                                                   ("junk", 1024, True), ("", 1024, False)])
def test_pool_pinned_cap_parser(value, want_mib, warns):
    """HDFS3_POOL_PINNED_MAX: digits with an optional K/M/G suffix; anything else keeps the 1 GiB
    default and says so on stderr instead of being read as a prefix of itself ("1.5G" was
    read as 1 byte). hdfs3_crc_pool_stats_get reports the cap without touching a GPU."""
    code = ("import ctypes, sys; sys.path.insert(0, %r)\n"
            "from libhdfs3_amd import _native\n"
            "st = _native.PoolStats(); assert _native.lib().hdfs3_crc_pool_stats_get(ctypes.byref(st)) == 0\n"
            "print(st.pinned_cap_bytes)\n") % REPO
    env = dict(os.environ, HDFS3_POOL_PINNED_MAX=value)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert int(out.stdout.strip().splitlines()[-1]) == want_mib << 20
    assert ("HDFS3_POOL_PINNED_MAX" in out.stderr) == warns, out.stderr
