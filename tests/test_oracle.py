"""CPU tests: pin the oracle (CPU restatement) to the reference's own fixtures.

- test/data/checksum1.in / checksum2.in, driven exactly as test/unit/TestChecksum.cpp:83-140
  (value-after-reset 0, every case at 8 alignments, streamed total);
- tests/golden/ref_hwcrc32c.* generated from the reference's HWCrc32c (make_golden.py);
- the verify-loop semantics of RemoteBlockReader.cpp:306-326 / LocalBlockReader.cpp:138-163.
"""
import json
import os

import numpy as np
import pytest

from util import (GOLDEN, HW, PCL, SW, fill_buffer, oracle, oracle_compute, oracle_crc, oracle_verify,
                  ptr, read_checksum1, read_checksum2, ref_lib, splitmix_bytes)

ENGINES = [SW, HW, PCL]
GOLD = np.load(os.path.join(GOLDEN, "ref_hwcrc32c.npz"))
META = json.load(open(os.path.join(GOLDEN, "ref_hwcrc32c.json")))


def update(engine, state, data: bytes):
    a = np.frombuffer(data, dtype=np.uint8)
    fn = [oracle().oracle_crc32c_sw_update, oracle().oracle_crc32c_hw_update,
          oracle().oracle_crc32c_pcl_update][engine]
    return fn(state, ptr(a) if a.nbytes else None, a.nbytes)


@pytest.mark.parametrize("engine", ENGINES)
def test_value_after_reset_is_zero(engine):
    # TestChecksum.cpp:87,103: getValue() after reset() is 0
    assert (~update(engine, 0xFFFFFFFF, b"")) & 0xFFFFFFFF == 0


@pytest.mark.parametrize("engine", ENGINES)
def test_checksum1_in_all_alignments(engine):
    cases = read_checksum1()
    assert len(cases) == 512 and cases[0] == (3251651376, b"a")
    for want, s in cases:
        buf = np.zeros(len(s) + 8, dtype=np.uint8)
        for j in range(8):  # TestChecksum.cpp:92-99
            buf[j:j + len(s)] = np.frombuffer(s, dtype=np.uint8)
            got = oracle().oracle_crc32c(engine, ptr(buf) + j, len(s))
            assert got == want, (engine, len(s), j)


@pytest.mark.parametrize("engine", ENGINES)
def test_checksum2_in_streamed(engine):
    result, lines = read_checksum2()
    assert result == 1963114415 and lines[0] == b"" and len(lines) == 512
    state = 0xFFFFFFFF
    for s in lines:  # TestChecksum.cpp:103-110
        state = update(engine, state, s)
    assert (~state) & 0xFFFFFFFF == result


@pytest.mark.parametrize("engine", ENGINES)
def test_all_lengths_all_alignments_vs_reference_fixture(engine):
    buf = splitmix_bytes(4096 + 8, META["seeds"]["lengths"])
    lens = GOLD["lengths"]
    for a in range(8):
        for n in list(range(0, 600)) + list(range(600, 4097, 37)) + [3071, 3072, 3073, 4095, 4096]:
            assert oracle().oracle_crc32c(engine, ptr(buf) + a, n) == lens[a, n], (engine, a, n)


def test_all_lengths_pcl_exhaustive():
    # the 3-way engine's block/remainder split is the only non-trivial control flow
    buf = splitmix_bytes(4096 + 8, META["seeds"]["lengths"])
    lens = GOLD["lengths"]
    for a in (0, 3, 7):
        got = [oracle().oracle_crc32c(PCL, ptr(buf) + a, n) for n in range(4097)]
        assert np.array_equal(np.array(got, dtype=np.uint32), lens[a])


@pytest.mark.parametrize("name", sorted(META["kat"]))
def test_survey_kats(name):
    inputs = {
        "off0_len512": fill_buffer(512, 0), "off512_len512": fill_buffer(512, 512),
        "off0_len2048": fill_buffer(2048, 0), "off0_len4096": fill_buffer(4096, 0),
        "str_123456789": np.frombuffer(b"123456789", np.uint8), "zeros512": np.zeros(512, np.uint8),
        "zeros2048": np.zeros(2048, np.uint8), "zeros4096": np.zeros(4096, np.uint8),
        "ff512": np.full(512, 0xFF, np.uint8),
    }
    for e in ENGINES:
        assert oracle_crc(inputs[name], e) == META["kat"][name]
    assert META["kat"]["off0_len512"] == 0x3D973599 and META["kat"]["str_123456789"] == 0xE3069283


def test_packet_fixture_compute_and_verify():
    pkt = splitmix_bytes(65536, META["seeds"]["packet"])
    crc = GOLD["pkt_crc"]
    for e in ENGINES:
        assert np.array_equal(oracle_compute(pkt, 512, e), crc)
    v = META["verify"]
    assert oracle_verify(pkt, 512, crc, False) == v["clean_remote"] == -1
    bad = pkt.copy()
    bad[META["packet"]["flip_byte"]] ^= META["packet"]["flip_mask"]
    assert oracle_verify(bad, 512, crc, False) == v["flip77_remote"] == 77
    assert oracle_verify(bad, 512, crc, True) == v["flip77_local"] == 77


def test_short_tail_semantics():
    # RemoteBlockReader.cpp:319 ignores a short tail mismatch; LocalBlockReader.cpp:149-161 does not
    pkt = splitmix_bytes(65536, META["seeds"]["packet"])
    n = META["packet"]["tail_len"]
    tail = GOLD["tail_crc"]
    assert np.array_equal(oracle_compute(pkt[:n], 512), tail)
    corrupt = tail.copy()
    corrupt[4 * 127] ^= 0xFF
    v = META["verify"]
    assert oracle_verify(pkt[:n], 512, tail, True) == v["tail_clean_local"] == -1
    assert oracle_verify(pkt[:n], 512, corrupt, False) == v["tail_corrupt_remote"] == -1
    assert oracle_verify(pkt[:n], 512, corrupt, True) == v["tail_corrupt_local"] == 127


@pytest.mark.parametrize("bpc", [512, 2048, 4096])
def test_bpc_fixture(bpc):
    big = splitmix_bytes(1 << 20, META["seeds"]["bpc"])
    assert np.array_equal(oracle_compute(big, bpc), GOLD[f"bpc{bpc}"])


def test_empty_and_tiny():
    e = np.zeros(0, dtype=np.uint8)
    assert oracle_compute(e, 512).nbytes == 0
    assert oracle_verify(e, 512, e, True) == -1
    one = np.frombuffer(b"a", np.uint8).copy()
    assert oracle_compute(one, 512).view(">u4")[0] == 0xC1D04330


def test_splitmix_numpy_matches_c():
    for n, seed in [(1, 1), (7, 2), (8, 3), (1000, 0x5EED), (4104, 0x5EED)]:
        a = np.zeros(n, dtype=np.uint8)
        oracle().oracle_fill_splitmix(ptr(a), n, seed)
        assert np.array_equal(a, splitmix_bytes(n, seed))


@pytest.mark.skipif(ref_lib() is None, reason="oracle/_ref not built (no /root/reference here)")
def test_oracle_vs_compiled_reference_random():
    ref = ref_lib()
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, 70000, dtype=np.uint8)
    for _ in range(400):
        a = int(rng.integers(0, 8))
        n = int(rng.integers(0, 69000))
        want = ref.ref_hw_crc32c(ptr(buf) + a, n)
        for e in ENGINES:
            assert oracle().oracle_crc32c(e, ptr(buf) + a, n) == want


def test_crc32_oracle_matches_zlib_and_check_value():
    """CHECKSUM_CRC32 (boost::crc_32_type behind Crc32.h:41-75): parity pinned by the
    standard check value and Python's zlib.crc32 (no reference test covers type 1)."""
    import zlib

    from util import oracle_compute_crc32, oracle_crc32

    assert oracle_crc32(b"123456789") == 0xCBF43926
    assert oracle_crc32(b"") == 0
    buf = splitmix_bytes(5000, 77)
    for n in list(range(0, 70)) + [511, 512, 513, 4095, 4096, 4097, 5000]:
        for off in (0, 3):
            piece = buf[off:off + n]
            assert oracle_crc32(piece) == zlib.crc32(piece.tobytes())
    words = oracle_compute_crc32(buf, 512)
    want = b"".join(zlib.crc32(buf[i:i + 512].tobytes()).to_bytes(4, "big") for i in range(0, buf.nbytes, 512))
    assert words.tobytes() == want
