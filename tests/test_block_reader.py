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


@pytest.mark.parametrize("bpc", [512, 4096, 8192, 12288, 16384, 20480, 65536])
def test_dense_batches_every_chunk_size(dn, bpc):
    """Round 5: batches land densely (the packets' words back to back, their data back to back from a
    4 KiB boundary) and verify as ONE contiguous block: the round kernel at 512 / 4096, the
    multi-round kernel at 8192 / 16384 / 65536, pieces + combine at 12288 (on the batch's own piece
    scratch). A whole block and a ranged read deliver the block's bytes; a flipped bit in the first,
    a middle and the last packet raises ChecksumException after EXACTLY the packets before it were
    delivered (RemoteBlockReader.cpp:306-326); a short tail's mismatch is ignored (:319)."""
    from libhdfs3_amd.engine import BlockReader
    from libhdfs3_amd._native import Hdfs3CrcError

    lb, port, add = dn
    per = max(bpc, 65536 // bpc * bpc)  # the loopback datanode's data bytes per packet
    n = 40 * per + bpc // 2 + 100  # 41 packets, the last one short with a short tail chunk
    data = splitmix_bytes(n, 5100 + bpc)
    bid = 50_000 + bpc
    crc = add(bid, data, bpc)
    out, st = _read(port, bid, 0, n, batch_packets=16)
    assert np.array_equal(out, data) and st["bytes_per_checksum"] == bpc and st["gpu_batches"] == 3
    start = 3 * per + 17
    out, _ = _read(port, bid, start, 20 * per, batch_packets=7)
    assert np.array_equal(out, data[start:start + 20 * per])
    tail = crc.copy()
    tail[-4] ^= 0x5A  # the short tail chunk's word: ignored by remote semantics
    add(bid + 1, data, bpc, crc=tail)
    out, _ = _read(port, bid + 1, 0, n, batch_packets=16)
    assert np.array_equal(out, data)
    for k, p in enumerate((0, 21, 39)):
        bad = data.copy()
        q = p * per + (per * 2) // 3
        bad[q] ^= 0x40
        add(bid + 2 + k, bad, bpc, crc=crc)
        with BlockReader("127.0.0.1", port, bid + 2 + k, 0, n, batch_packets=16) as r:
            got = np.zeros(n, np.uint8)
            pos = 0
            with pytest.raises(Hdfs3CrcError) as ei:
                while True:
                    g = r.read_into(got, pos, min(1 << 20, n - pos))
                    assert g > 0
                    pos += g
            assert ei.value.rc == -errno.EIO and "ChecksumException" in str(ei.value)
        assert pos == p * per, (p, pos)
        assert np.array_equal(got[:pos], data[:pos])


_WIRE_CHILD = r"""
import sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/tests"]
from loopback import LoopbackDatanode
from util import oracle_compute, splitmix_bytes
from libhdfs3_amd.engine import BlockReader
dn = LoopbackDatanode()
try:
    for bpc in (512, 4096, 8192):
        data = splitmix_bytes((6 << 20) + 333, bpc)
        crc = oracle_compute(data, bpc)
        dn.add_block(bpc, data, crc, bpc)
        with BlockReader("127.0.0.1", dn.port, bpc, 0, data.nbytes, batch_packets=16) as r:
            assert np.array_equal(r.read_all(data.nbytes), data)
        bad = data.copy()
        bad[(5 << 20) + 9] ^= 1
        dn.add_block(bpc + 1, bad, crc, bpc)
        try:
            with BlockReader("127.0.0.1", dn.port, bpc + 1, 0, data.nbytes, batch_packets=16) as r:
                r.read_all(data.nbytes)
            print("NO EXCEPTION", bpc)
        except Exception as e:
            assert "ChecksumException" in str(e), e
        print("ok", bpc)
finally:
    dn.stop()
"""


def test_wire_layout_knob_keeps_the_packet_kernels():
    """HDFS3_READER_LAYOUT=wire (read once per process: a child) keeps the round-4 wire layout and
    its packet kernels (pitch walk / segmented / chunk-per-lane): same bytes and the same exception."""
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HDFS3_READER_LAYOUT="wire")
    out = subprocess.run([sys.executable, "-c", _WIRE_CHILD, repo], env=env, capture_output=True, text=True,
                         timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split() == ["ok", "512", "ok", "4096", "ok", "8192"], out.stdout


def test_dense_batches_of_large_packets_keep_the_arena_size():
    """256 KiB datanode packets (64-packet batches would need 16 MiB): a dense batch closes when the
    arena the ring was sized for is full, as the wire layout does, instead of growing it (the pinned
    pool's budget assumes 64 KiB packets): 15 packets per batch, every byte delivered."""
    from loopback import LoopbackDatanode

    node = LoopbackDatanode(packet_bytes=256 << 10)
    try:
        data = splitmix_bytes(16 << 20, 4321)
        node.add_block(1, data, oracle_compute(data, 512), 512)
        out, st = _read(node.port, 1, 0, data.nbytes, batch_packets=64)
        assert np.array_equal(out, data)
        # 15 packets per batch in a 64 x 66,064-byte arena (fewer batches if the pooled ctx hands back a
        # larger cached arena; a batch grown to take all 64 packets would be one)
        assert st["packets"] == 64 and st["gpu_batches"] >= 2, st
    finally:
        node.stop()
