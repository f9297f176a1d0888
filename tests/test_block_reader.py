"""GPU tests of the read-path drop-in: hdfs3_block_reader (RemoteBlockReader with batched GPU
verify) against the loopback datanode. Reference semantics checked: delivered bytes are the
block bytes of [start, start+len); a full-chunk CRC mismatch raises ChecksumException (-EIO)
after the packets before it were delivered (RemoteBlockReader.cpp:306-326); a short tail
mismatch is ignored (:319); CHECKSUM_OK is sent only after every packet verified (:289-304);
verify=false reads without checking (InputStream verify flag)."""
import errno

import numpy as np
import pytest

from util import oracle_compute, splitmix_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dn():
    from loopback import LoopbackDatanode

    node = LoopbackDatanode()

    def add(block_id, data, bpc, crc=None, ctype=2):
        crc = oracle_compute(data, bpc) if crc is None else crc
        node.add_block(block_id, data, crc, bpc, ctype)
        return crc

    yield node, node.port, add
    node.stop()


def _read(port, block_id, start, length, **kw):
    from libhdfs3_amd.engine import BlockReader

    with BlockReader("127.0.0.1", port, block_id, start, length, **kw) as r:
        out = r.read_all(length)
        return out, r.stats()


@pytest.mark.parametrize("bpc,batch", [(512, 64), (512, 3), (4096, 5), (2048, 1)])
def test_full_block_verified_read(dn, bpc, batch):
    lb, port, add = dn
    data = splitmix_bytes(8 << 20, bpc + batch)
    add(1000 + bpc + batch, data, bpc)
    out, st = _read(port, 1000 + bpc + batch, 0, data.nbytes, batch_packets=batch)
    assert np.array_equal(out, data)
    assert st["bytes_per_checksum"] == bpc and st["gpu_batches"] >= st["packets"] // batch


def test_ranged_reads_and_short_tail_block(dn):
    lb, port, add = dn
    data = splitmix_bytes(3_000_000 + 123, 42)  # last chunk short
    add(2000, data, 512)
    for start, length in [(0, 1), (1, 1000), (511, 2), (65535, 70000), (777_777, 1_234_567),
                          (data.nbytes - 1000, 1000), (0, data.nbytes)]:
        out, _ = _read(port, 2000, start, length, batch_packets=7)
        assert np.array_equal(out, data[start:start + length]), (start, length)


def test_corruption_raises_checksum_exception_after_good_packets(dn):
    from libhdfs3_amd.engine import BlockReader
    from libhdfs3_amd._native import Hdfs3CrcError

    lb, port, add = dn
    data = splitmix_bytes(4 << 20, 77)
    crc = oracle_compute(data, 512)
    bad = data.copy()
    bad_pos = 37 * 65536 + 1000  # packet 37 (64 KiB packets)
    bad[bad_pos] ^= 0x10
    add(3000, bad, 512, crc=crc)
    with BlockReader("127.0.0.1", port, 3000, 0, data.nbytes, batch_packets=16) as r:
        out = np.zeros(data.nbytes, np.uint8)
        pos = 0
        with pytest.raises(Hdfs3CrcError) as ei:
            while True:
                got = r.read_into(out, pos, 1 << 20)
                assert got > 0
                pos += got
        assert ei.value.rc == -errno.EIO and "ChecksumException" in str(ei.value)
    # every byte delivered before the exception is good and precedes the bad packet
    assert pos <= 37 * 65536 and pos >= 32 * 65536
    assert np.array_equal(out[:pos], data[:pos])


def test_short_tail_mismatch_is_ignored_like_remote_reader(dn):
    lb, port, add = dn
    data = splitmix_bytes(200_000 + 100, 5)
    crc = oracle_compute(data, 512)
    crc[-4] ^= 0xFF  # the short tail chunk's stored CRC
    add(4000, data, 512, crc=crc)
    out, _ = _read(port, 4000, 0, data.nbytes)
    assert np.array_equal(out, data)


def test_verify_disabled_delivers_corrupt_bytes(dn):
    lb, port, add = dn
    data = splitmix_bytes(1 << 20, 6)
    crc = oracle_compute(data, 512)
    bad = data.copy()
    bad[12345] ^= 1
    add(5000, bad, 512, crc=crc)
    out, _ = _read(port, 5000, 0, data.nbytes, verify=False)
    assert np.array_equal(out, bad)


def test_checksum_ok_status_sent_after_verified_read(dn):
    lb, port, add = dn
    data = splitmix_bytes(1 << 20, 8)
    add(6000, data, 512)
    out, _ = _read(port, 6000, 0, data.nbytes)
    assert np.array_equal(out, data)
    assert lb.last_status(wait_for=6) == 6


def test_unknown_block_fails_open(dn):
    from libhdfs3_amd.engine import BlockReader
    from libhdfs3_amd._native import Hdfs3CrcError

    lb, port, add = dn
    with pytest.raises(Hdfs3CrcError):
        BlockReader("127.0.0.1", port, 987654, 0, 100)


def test_checksum_null_block_reads_without_verify(dn):
    lb, port, add = dn
    data = splitmix_bytes(300_000, 9)
    lb.add_block(7000, data, None, 512, ctype=0)  # CHECKSUM_NULL: no CRC words on the wire
    out, st = _read(port, 7000, 0, data.nbytes)
    assert np.array_equal(out, data) and st["bytes_per_checksum"] == 512


def test_crc32_type_block_is_verified_with_the_zlib_polynomial(dn):
    from libhdfs3_amd.engine import BlockReader
    from libhdfs3_amd._native import Hdfs3CrcError
    from util import oracle_compute_crc32

    lb, port, add = dn
    data = splitmix_bytes(2_000_000 + 5, 10)
    crc = oracle_compute_crc32(data, 512)
    lb.add_block(7001, data, crc, 512, ctype=1)  # CHECKSUM_CRC32
    out, st = _read(port, 7001, 0, data.nbytes)
    assert np.array_equal(out, data)
    bad = data.copy()
    bad[1_000_000] ^= 2
    lb.add_block(7002, bad, crc, 512, ctype=1)
    with BlockReader("127.0.0.1", port, 7002, 0, data.nbytes) as r:
        with pytest.raises(Hdfs3CrcError):
            r.read_all(data.nbytes)
    # CRC32C words under a CRC32 response must fail (the polynomial follows the response)
    lb.add_block(7003, data, oracle_compute(data, 512), 512, ctype=1)
    with BlockReader("127.0.0.1", port, 7003, 0, data.nbytes) as r:
        with pytest.raises(Hdfs3CrcError):
            r.read_all(data.nbytes)


def test_datanode_drop_mid_block_is_an_io_error(dn):
    from libhdfs3_amd.engine import BlockReader
    from libhdfs3_amd._native import Hdfs3CrcError
    from loopback import LoopbackDatanode

    node = LoopbackDatanode()
    try:
        data = splitmix_bytes(2 << 20, 11)
        node.add_block(1, data, oracle_compute(data, 512), 512)
        node.set_fail_after(1 << 20)
        with BlockReader("127.0.0.1", node.port, 1, 0, data.nbytes, timeout_ms=5000) as r:
            out = np.zeros(data.nbytes, np.uint8)
            pos = 0
            with pytest.raises(Hdfs3CrcError):
                while True:
                    got = r.read_into(out, pos, 1 << 16)
                    assert got > 0
                    pos += got
            assert pos <= 1 << 20 and np.array_equal(out[:pos], data[:pos])
    finally:
        node.stop()
