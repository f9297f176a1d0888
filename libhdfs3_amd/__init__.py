"""libhdfs3_amd — MI355X-native per-chunk CRC32C engine for libhdfs3's checksum hot path.

The product is the C-ABI shared library libhdfs3_amd/lib/libhdfs3_crc.so
(include/hdfs3_crc.h) built from libhdfs3_amd/csrc/ (hand-written gfx950 HIP
kernels + C++ host layer). This Python package is a thin ctypes handle over it
for tests and bench.py; it has no compute path of its own.
"""
from ._native import Hdfs3CrcError, LIB_PATH  # noqa: F401

__all__ = ["Hdfs3CrcError", "LIB_PATH"]
