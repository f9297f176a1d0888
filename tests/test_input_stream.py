"""GPU tests of the hdfsRead/hdfsPread/hdfsSeek surface (hdfs3_input_stream) over loopback
datanodes acting as replicas. Reference behaviour checked (src/client/InputStreamImpl.cpp):
read never crosses a block boundary (readOneBlock :616-712); a ChecksumException or I/O
failure moves to the next replica not yet failed (:682-708, choseBestNode :322-335); when
every replica failed the call fails with EIO (:369-383 -> Hdfs.cpp handleException); pread
reads across blocks without moving the cursor and returns -1 outside the file (:815-860);
seek past EOF is EOVERFLOW (HdfsEndOfStream, Hdfs.cpp:276-277); read at EOF returns 0."""
import errno

import numpy as np
import pytest

from util import oracle_compute, splitmix_bytes

pytestmark = pytest.mark.gpu

BPC = 512
SIZES = [3 << 20, 3 << 20, 1_000_000 + 77]  # ragged last block, short last chunk


@pytest.fixture(scope="module")
def cluster():
    """Two healthy replicas of a 3-block file, plus the file's bytes."""
    from loopback import LoopbackDatanode

    a, b = LoopbackDatanode(), LoopbackDatanode()
    blocks, parts = [], []
    for i, n in enumerate(SIZES):
        d = splitmix_bytes(n, 100 + i)
        c = oracle_compute(d, BPC)
        for node in (a, b):
            node.add_block(500 + i, d, c, BPC)
        blocks.append((500 + i, n))
        parts.append(d)
    yield a, b, blocks, np.concatenate(parts)
    a.stop()
    b.stop()


def _stream(blocks, replicas, **kw):
    from libhdfs3_amd.engine import InputStream

    return InputStream([(bid, n, replicas) for bid, n in blocks], **kw)


def test_sequential_read_walks_blocks(cluster):
    a, b, blocks, whole = cluster
    with _stream(blocks, [("127.0.0.1", a.port)]) as s:
        assert s.length == whole.nbytes
        out = np.empty(whole.nbytes, np.uint8)
        pos = 0
        while pos < whole.nbytes:
            n = s.read_into(out, pos, min(5 << 20, whole.nbytes - pos))
            assert n > 0
            # readOneBlock never returns bytes of two blocks
            starts = np.cumsum([0] + SIZES)
            blk = np.searchsorted(starts, pos, side="right") - 1
            assert pos + n <= starts[blk + 1]
            pos += n
            assert s.tell() == pos
        assert pos == whole.nbytes and np.array_equal(out, whole)
        assert s.read_into(np.zeros(10, np.uint8)) == 0  # EOF
        assert s.stats()["readers_opened"] == 3 and s.stats()["failovers"] == 0


def test_pread_across_blocks_keeps_cursor(cluster):
    from libhdfs3_amd.engine import HdfsIOError

    a, b, blocks, whole = cluster
    with _stream(blocks, [("127.0.0.1", a.port)]) as s:
        s.seek(12345)
        for pos, n in [(0, 1), (SIZES[0] - 10, 20), (SIZES[0] - 1, SIZES[1] + 2), (whole.nbytes - 5, 100),
                       (777, 5 << 20)]:
            out = np.zeros(n, np.uint8)
            got = s.pread_into(pos, out)
            want = whole[pos:pos + n]
            assert got == want.nbytes and np.array_equal(out[:got], want)
        assert s.tell() == 12345
        with pytest.raises(HdfsIOError) as ei:
            s.pread_into(whole.nbytes, np.zeros(4, np.uint8))
        assert ei.value.errno == errno.EINVAL


def test_seek_skip_and_reopen(cluster):
    from libhdfs3_amd.engine import HdfsIOError

    a, b, blocks, whole = cluster
    with _stream(blocks, [("127.0.0.1", a.port)]) as s:
        buf = np.zeros(1000, np.uint8)
        s.read_into(buf)
        opened = s.stats()["readers_opened"]
        s.seek(1000 + 100_000)  # small forward seek: skip through the open reader
        assert s.read_into(buf) > 0 and np.array_equal(buf, whole[101_000:102_000])
        assert s.stats()["readers_opened"] == opened
        for pos in [50, SIZES[0] + 3, whole.nbytes - 10]:  # backward / other block / near EOF
            s.seek(pos)
            n = s.read_into(buf, 0, 10)
            assert n == 10 and np.array_equal(buf[:10], whole[pos:pos + 10])
        s.seek(whole.nbytes)
        assert s.read_into(buf, 0, 10) == 0
        with pytest.raises(HdfsIOError) as ei:
            s.seek(whole.nbytes + 1)
        assert ei.value.errno == errno.EOVERFLOW


def test_checksum_failure_fails_over_to_next_replica(cluster):
    from loopback import LoopbackDatanode

    a, b, blocks, whole = cluster
    bad = LoopbackDatanode()
    try:
        for i, (bid, n) in enumerate(blocks):
            d = whole[sum(SIZES[:i]):sum(SIZES[:i]) + n]
            c = oracle_compute(d, BPC)
            if i == 1:
                d = d.copy()
                d[2_000_000] ^= 0x40  # corrupt replica of block 1
            bad.add_block(bid, d, c, BPC)
        with _stream(blocks, [("127.0.0.1", bad.port), ("127.0.0.1", b.port)]) as s:
            got = s.read_fully(whole.nbytes)
            assert np.array_equal(got, whole)
            st = s.stats()
            assert st["failovers"] == 1 and st["readers_opened"] == 4
        # pread over the corrupt region fails over as well
        with _stream(blocks, [("127.0.0.1", bad.port), ("127.0.0.1", b.port)]) as s:
            out = np.zeros(1 << 20, np.uint8)
            pos = SIZES[0] + 1_500_000
            assert s.pread_into(pos, out) == out.nbytes
            assert np.array_equal(out, whole[pos:pos + out.nbytes])
            assert s.stats()["failovers"] == 1
    finally:
        bad.stop()


def test_every_replica_bad_is_eio_after_good_bytes(cluster):
    from libhdfs3_amd.engine import HdfsIOError
    from loopback import LoopbackDatanode

    a, b, blocks, whole = cluster
    bad = LoopbackDatanode()
    try:
        d = whole[:SIZES[0]].copy()
        c = oracle_compute(d, BPC)
        d[100_000] ^= 1
        bad.add_block(blocks[0][0], d, c, BPC)
        with _stream(blocks[:1], [("127.0.0.1", bad.port)]) as s:
            out = np.zeros(SIZES[0], np.uint8)
            pos = 0
            with pytest.raises(HdfsIOError) as ei:
                while True:
                    n = s.read_into(out, pos, 1 << 20)
                    assert n > 0
                    pos += n
            assert ei.value.errno == errno.EIO
            assert "all nodes have been tried" in str(ei.value)
            assert pos <= 100_000 and np.array_equal(out[:pos], whole[:pos])
    finally:
        bad.stop()


def test_dropped_connection_and_dead_node_fail_over(cluster):
    from loopback import LoopbackDatanode

    a, b, blocks, whole = cluster
    flaky, dead = LoopbackDatanode(), LoopbackDatanode()
    dead_port = dead.port
    dead.stop()  # nothing listens there any more
    try:
        off = 0
        for bid, n in blocks:
            d = whole[off:off + n]
            flaky.add_block(bid, d, oracle_compute(d, BPC), BPC)
            off += n
        flaky.set_fail_after(1 << 20)
        reps = [("127.0.0.1", dead_port), ("127.0.0.1", flaky.port), ("127.0.0.1", a.port)]
        with _stream(blocks, reps, timeout_ms=5000) as s:
            got = s.read_fully(whole.nbytes)
            assert np.array_equal(got, whole)
            # the flaky node drops blocks 0 and 1 after 1 MiB (block 2 is shorter); the dead
            # node fails at connect, which setupBlockReader handles without a read failover
            assert s.stats()["failovers"] == 2
    finally:
        flaky.stop()
