"""GPU parity of CHECKSUM_CRC32 (zlib polynomial; boost::crc_32_type behind Crc32.h:41-75),
selected per ctx with hdfs3_crc_ctx_set_checksum_type. The same kernels run with the CRC-32
table and fold images, so every kernel variant is checked against the bit-serial oracle
(tests/util.oracle_compute_crc32) and zlib. Parity unpinned by reference tests (none cover
type 1): pinned by the standard check value and zlib."""
import zlib

import numpy as np
import pytest

from util import oracle_compute, oracle_compute_crc32, splitmix_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx32():
    from libhdfs3_amd.engine import CrcContext

    c = CrcContext(0)
    c.set_checksum_type(1)
    assert c.checksum_type == 1
    yield c
    c.close()


def test_check_value_and_type_switch(ctx32):
    from libhdfs3_amd.engine import CrcContext
    from libhdfs3_amd._native import Hdfs3CrcError

    s = np.frombuffer(b"123456789", np.uint8)
    assert ctx32.compute(s, 4096).view(">u4")[0] == 0xCBF43926
    c = CrcContext(0)
    assert c.checksum_type == 2
    assert c.compute(s, 4096).view(">u4")[0] == 0xE3069283
    c.set_checksum_type(1)
    assert c.compute(s, 4096).view(">u4")[0] == 0xCBF43926
    c.set_checksum_type(2)
    assert c.compute(s, 4096).view(">u4")[0] == 0xE3069283
    with pytest.raises(Hdfs3CrcError):
        c.set_checksum_type(0)
    c.close()


@pytest.mark.parametrize("bpc", [512, 1024, 2048, 4096, 8192, 65536])
def test_ragged_lengths_host_and_device(ctx32, bpc):
    from libhdfs3_amd.engine import DeviceBuffer

    for n in [1, bpc - 1, bpc, 4096 * 9 + 13, 4096 * 256 * 3 + bpc + 7, (1 << 22) + 3]:
        data = splitmix_bytes(n, bpc * 31 + n)
        want = oracle_compute_crc32(data, bpc)
        assert np.array_equal(ctx32.compute(data, bpc), want), (bpc, n)
        d = ctx32.upload(data)
        dc = DeviceBuffer(want.nbytes)
        ctx32.compute_dev(d.ptr, n, bpc, dc.ptr)
        assert np.array_equal(ctx32.download(dc, want.nbytes), want), (bpc, n)
        assert ctx32.verify_dev(d.ptr, n, bpc, dc.ptr, True) == -1
        # a CRC32C word list must not pass a CRC32 verify
        if n >= bpc:
            assert ctx32.verify(data, bpc, oracle_compute(data, bpc), False) == 0
    first = splitmix_bytes(3 * bpc, 5)
    assert ctx32.compute(first, bpc)[:4].view(">u4")[0] == zlib.crc32(first[:bpc].tobytes())


@pytest.mark.parametrize("variant", [0, 92, 93, 94, 95])
@pytest.mark.parametrize("bpc", [512, 4096])
def test_every_kernel_variant_crc32(lab_ctx, variant, bpc):
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import DeviceBuffer

    lib = _native.lab()
    ctx32 = lab_ctx
    try:
        ctx32.set_checksum_type(1)
        lib.hdfs3x_set_variant(variant)
        for n in (4096 * 37, 4096 * 300 + bpc * 2 + 77):
            data = splitmix_bytes(n, variant * 7 + bpc + n)
            want = oracle_compute_crc32(data, bpc)
            d = ctx32.upload(data)
            dc = DeviceBuffer(want.nbytes)
            ctx32.compute_dev(d.ptr, n, bpc, dc.ptr)
            assert np.array_equal(ctx32.download(dc, want.nbytes), want), (variant, bpc, n)
            nc = (n + bpc - 1) // bpc
            for k in (0, nc // 2):
                pos = k * bpc + 3
                ctx32.upload(np.array([data[pos] ^ 8], np.uint8), d, offset=pos)
                assert ctx32.verify_dev(d.ptr, n, bpc, dc.ptr, False) == k
                ctx32.upload(data[pos:pos + 1], d, offset=pos)
    finally:
        lib.hdfs3x_set_variant(0)
        ctx32.set_checksum_type(2)


def test_packets_api_crc32(ctx32):
    bpc = 512
    pk, parts, off = [], [], 0
    for i, n in enumerate([65536, 65536 - 100, 777, 512]):
        data = splitmix_bytes(n, 40 + i)
        crc = oracle_compute_crc32(data, bpc)
        pad = (-(off + crc.nbytes)) % 16
        parts += [np.zeros(pad, np.uint8), crc, data]
        pk.append((off + pad + crc.nbytes, off + pad, n))
        off += pad + crc.nbytes + n
    arena = np.concatenate(parts)
    assert ctx32.verify_packets(arena, pk, bpc) == (-1, -1)
    bad = arena.copy()
    bad[pk[2][0] + 600] ^= 1  # packet 2, chunk 1 = its short tail: remote semantics ignore it
    assert ctx32.verify_packets(bad, pk, bpc) == (-1, -1)
    assert ctx32.verify_packets(bad, pk, bpc, check_short_tail=True) == (2, 1)
