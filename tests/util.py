"""Shared test helpers: the oracle binding (test infrastructure) and deterministic data.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg touch oracle/.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import c_double, c_int, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")
REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_hwcrc32c.so")

SW, HW, PCL = 0, 1, 2


def _build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all"], check=True)


_ORACLE = None


def oracle() -> ctypes.CDLL:
    """The CPU restatement (oracle/crc32c_oracle.c) — the parity checker."""
    global _ORACLE
    if _ORACLE is None:
        if not os.path.exists(ORACLE_SO):
            _build_oracle()
        lib = ctypes.CDLL(ORACLE_SO)
        lib.oracle_crc32c_sw_update.restype = c_uint32
        lib.oracle_crc32c_sw_update.argtypes = [c_uint32, c_void_p, c_size_t]
        lib.oracle_crc32c_hw_update.restype = c_uint32
        lib.oracle_crc32c_hw_update.argtypes = [c_uint32, c_void_p, c_size_t]
        lib.oracle_crc32c_pcl_update.restype = c_uint32
        lib.oracle_crc32c_pcl_update.argtypes = [c_uint32, c_void_p, c_size_t]
        lib.oracle_crc32c.restype = c_uint32
        lib.oracle_crc32c.argtypes = [c_int, c_void_p, c_size_t]
        lib.oracle_compute_chunks.restype = None
        lib.oracle_compute_chunks.argtypes = [c_int, c_void_p, c_size_t, c_uint32, c_void_p]
        lib.oracle_verify_chunks.restype = c_int64
        lib.oracle_verify_chunks.argtypes = [c_int, c_void_p, c_size_t, c_uint32, c_void_p, c_int]
        lib.oracle_bench_verify.restype = c_double
        lib.oracle_bench_verify.argtypes = [c_int, c_void_p, c_size_t, c_uint32, c_void_p, c_int, c_int,
                                            ctypes.POINTER(c_int64)]
        lib.oracle_crc32_update.restype = c_uint32
        lib.oracle_crc32_update.argtypes = [c_uint32, c_void_p, c_size_t]
        lib.oracle_compute_chunks_crc32.restype = None
        lib.oracle_compute_chunks_crc32.argtypes = [c_void_p, c_size_t, c_uint32, c_void_p]
        lib.oracle_fill_splitmix.restype = None
        lib.oracle_fill_splitmix.argtypes = [c_void_p, c_size_t, c_uint64]
        _ORACLE = lib
    return _ORACLE


def ref_lib() -> ctypes.CDLL | None:
    """The reference's own HWCrc32c (oracle/_ref), when it was built in this container."""
    if not os.path.exists(REF_SO):
        return None
    lib = ctypes.CDLL(REF_SO)
    lib.ref_hw_crc32c.restype = c_uint32
    lib.ref_hw_crc32c.argtypes = [c_void_p, c_int]
    lib.ref_hw_verify.restype = c_int64
    lib.ref_hw_verify.argtypes = [c_void_p, c_int64, c_int, c_void_p, c_int]
    lib.ref_hw_bench_verify.restype = c_double
    lib.ref_hw_bench_verify.argtypes = [c_void_p, c_int64, c_int, c_void_p, c_int, c_int, ctypes.POINTER(c_int64)]
    lib.ref_hw_available.restype = c_int
    return lib


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ---- deterministic data (same stream as oracle_fill_splitmix) --------------------

_GOLDEN_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix_bytes(n: int, seed: int) -> np.ndarray:
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(1, words + 1, dtype=np.uint64) * _GOLDEN_GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def fill_buffer(n: int, offset: int = 0) -> np.ndarray:
    """mock/TestUtil.h:44-53 FillBuffer: repeating "012345678\\n" from `offset`."""
    pat = np.frombuffer(b"012345678\n", dtype=np.uint8)
    idx = (np.arange(n, dtype=np.int64) + offset) % 10
    return pat[idx].copy()


def oracle_compute(data: np.ndarray, bpc: int, engine: int = PCL) -> np.ndarray:
    n = (data.nbytes + bpc - 1) // bpc
    out = np.zeros(4 * n, dtype=np.uint8)
    oracle().oracle_compute_chunks(engine, ptr(data) if data.nbytes else None, data.nbytes, bpc, ptr(out))
    return out


def oracle_compute_crc32(data: np.ndarray, bpc: int) -> np.ndarray:
    """CHECKSUM_CRC32 words (zlib polynomial) per chunk, big-endian."""
    n = (data.nbytes + bpc - 1) // bpc
    out = np.zeros(4 * n, dtype=np.uint8)
    oracle().oracle_compute_chunks_crc32(ptr(data) if data.nbytes else None, data.nbytes, bpc, ptr(out))
    return out


def oracle_crc32(data: bytes | np.ndarray) -> int:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return (~int(oracle().oracle_crc32_update(0xFFFFFFFF, ptr(a) if a.nbytes else None, a.nbytes))) & 0xFFFFFFFF


def oracle_verify(data: np.ndarray, bpc: int, crc_be: np.ndarray, check_short_tail: bool,
                  engine: int = PCL) -> int:
    return int(oracle().oracle_verify_chunks(engine, ptr(data) if data.nbytes else None, data.nbytes, bpc,
                                             ptr(crc_be) if crc_be.nbytes else None, int(check_short_tail)))


def oracle_crc(data: bytes | np.ndarray, engine: int = PCL) -> int:
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return int(oracle().oracle_crc32c(engine, ptr(a) if a.nbytes else None, a.nbytes))


def read_checksum1():
    """test/data/checksum1.in as parsed by TestChecksum::SetUp (TestChecksum.cpp:46-59)."""
    cases = []
    with open(os.path.join(GOLDEN, "checksum1.in"), "rb") as f:
        for line in f.read().split(b"\n"):
            if not line:
                continue
            v, s = line.split(b" ", 1)
            cases.append((int(v), s.split()[0]))
    return cases


def read_checksum2():
    """test/data/checksum2.in (TestChecksum.cpp:61-70): expected total, then lines fed
    streaming; getline after `in >> result` yields an initial empty string."""
    with open(os.path.join(GOLDEN, "checksum2.in"), "rb") as f:
        raw = f.read()
    first_nl = raw.index(b"\n")
    result = int(raw[:first_nl].split()[0])
    rest = raw[:first_nl][len(raw[:first_nl].split()[0]):]
    lines = [rest] + raw[first_nl + 1:].split(b"\n")
    if lines and lines[-1] == b"":
        lines = lines[:-1]
    return result, lines
