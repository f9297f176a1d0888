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


# --- the reference's own function-test shape (test/function/TestInputStream.cpp) -------------
# Files hold the FillBuffer "012345678\n" pattern and are written with 1 KiB packets
# (TestInputStream.cpp:62 output.default.packetsize=1024), so every read-path packet carries
# two 512 B chunks; reads are checked with CheckBuffer at their file offset.

def _fill_cluster(sizes, packet_bytes, base_id, bpc=BPC):
    from loopback import LoopbackDatanode

    from util import fill_buffer

    node = LoopbackDatanode(packet_bytes=packet_bytes)
    blocks, off = [], 0
    for i, n in enumerate(sizes):
        d = fill_buffer(n, off)
        node.add_block(base_id + i, d, oracle_compute(d, bpc), bpc)
        blocks.append((base_id + i, n))
        off += n
    return node, blocks


@pytest.mark.parametrize("packet_bytes", [1024, 512, 1536])
def test_reference_checksum_read_pattern_1k_packets(packet_bytes):
    """TestInputStream.cpp:126-154 CheckSum: reads of size, size-100 and size+100 bytes at a
    running offset, each checked against FillBuffer; 40 KiB file (largefile, :97-101) split
    into 2 KiB blocks so reads cross block boundaries the way readOneBlock cuts them."""
    from util import fill_buffer

    total = 20 * 2048
    node, blocks = _fill_cluster([2048] * 20, packet_bytes, 700)
    try:
        with _stream(blocks, [("127.0.0.1", node.port)]) as s:
            pos = 0
            for want in [1024, 924, 1124] * 40:
                if pos >= total:
                    break
                buf = np.zeros(want, np.uint8)
                got = 0
                while got < want and pos + got < total:  # readFully over block cuts
                    n = s.read_into(buf, got, want - got)
                    assert n > 0
                    got += n
                assert np.array_equal(buf[:got], fill_buffer(got, pos))
                pos += got
            assert pos == total and s.read_into(np.zeros(8, np.uint8)) == 0
            assert s.stats()["failovers"] == 0
    finally:
        node.stop()


@pytest.mark.parametrize("size", [512, 1024, 2048])
def test_reference_read_fully_sizes(size):
    """TestInputStream.cpp:194-205 ReadFully(size), (size-100), (size+100) from offset 0 of a
    file served in 1 KiB packets; the short last chunk is verified too."""
    from util import fill_buffer

    node, blocks = _fill_cluster([size + 100], 1024, 760)
    try:
        for n in (size, size - 100, size + 100):
            with _stream(blocks, [("127.0.0.1", node.port)]) as s:
                got = s.read_fully(n)
                assert np.array_equal(got, fill_buffer(n, 0))
    finally:
        node.stop()


def test_reference_checksum_corruption_1k_packets():
    """A flipped byte inside a 1 KiB packet: the corrupt replica raises the ChecksumException
    path (failover to the good replica, RemoteBlockReader.cpp:306-326 -> InputStreamImpl.cpp
    :682-708); with the corrupt replica alone the read fails with EIO after the good bytes."""
    from libhdfs3_amd.engine import HdfsIOError
    from loopback import LoopbackDatanode

    from util import fill_buffer

    total = 64 << 10
    good, blocks = _fill_cluster([total], 1024, 780)
    bad = LoopbackDatanode(packet_bytes=1024)
    try:
        d = fill_buffer(total, 0)
        c = oracle_compute(d, BPC)
        d = d.copy()
        d[40_000] ^= 0x01  # chunk 78, packet 39
        bad.add_block(780, d, c, BPC)
        with _stream(blocks, [("127.0.0.1", bad.port), ("127.0.0.1", good.port)]) as s:
            assert np.array_equal(s.read_fully(total, chunk=3000), fill_buffer(total, 0))
            assert s.stats()["failovers"] == 1
        with _stream(blocks, [("127.0.0.1", bad.port)]) as s:
            out = np.zeros(total, np.uint8)
            pos = 0
            with pytest.raises(HdfsIOError) as ei:
                while True:
                    n = s.read_into(out, pos, 3000)
                    assert n > 0
                    pos += n
            assert ei.value.errno == errno.EIO
            assert pos <= 78 * BPC and np.array_equal(out[:pos], fill_buffer(pos, 0))
    finally:
        good.stop()
        bad.stop()


def _check_file_content(blocks, port, length, errors):
    """TestInputStream.cpp:256-273 CheckFileContent: 20 KiB + 1 reads, CheckBuffer each."""
    from util import fill_buffer

    try:
        with _stream(blocks, [("127.0.0.1", port)]) as s:
            buf = np.zeros(20 * 1024 + 1, np.uint8)
            off = 0
            while off < length:
                n = s.read_into(buf, 0, min(buf.nbytes, length - off))
                assert n > 0
                if not np.array_equal(buf[:n], fill_buffer(n, off)):
                    errors.append(f"mismatch at {off}")
                    return
                off += n
    except Exception as e:  # noqa: BLE001 - collected and asserted by the caller
        errors.append(repr(e))


def test_reference_read_one_file_same_time():
    """TestInputStream.cpp:299-319 TestReadOneFileSameTime (scaled: 16 threads instead of 50,
    an 8 MiB + 234 B file instead of 1 GiB): concurrent streams, each with its own engine
    context, read the first 1 MiB + 234 B of one file through 1 KiB packets."""
    import threading

    size = (8 << 20) + 234
    node, blocks = _fill_cluster([4 << 20, 4 << 20, 234], 1024, 800)
    errors: list = []
    try:
        ts = [threading.Thread(target=_check_file_content, args=(blocks, node.port, (1 << 20) + 234, errors))
              for _ in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in ts), "reader thread hung"
        assert not errors, errors[:3]
        assert sum(n for _, n in blocks) == size
    finally:
        node.stop()


def test_reference_read_many_files_same_time():
    """TestInputStream.cpp:321-342 TestReadManyFileSameTime (scaled: 8 files of 2 MiB + 234 B
    on separate datanodes, one thread per file)."""
    import threading

    nodes, errors = [], []
    try:
        for i in range(8):
            nodes.append(_fill_cluster([1 << 20, (1 << 20) + 234], 1024, 900 + 10 * i))
        ts = [threading.Thread(target=_check_file_content, args=(blocks, node.port, (1 << 20) + 234, errors))
              for node, blocks in nodes]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in ts), "reader thread hung"
        assert not errors, errors[:3]
    finally:
        for node, _ in nodes:
            node.stop()


def test_config5_1gib_file_at_size():
    """BASELINE.json configs[4]: hdfs3_input_read of a 1 GiB file (8 x 128 MiB blocks, 64 KiB
    packets) from loopback datanodes. Stored words come from the oracle; the bytes read must
    equal the source; with a corrupted replica listed first for block 5 the stream fails over
    exactly once and still returns every byte."""
    from loopback import LoopbackDatanode

    nblk, bs = 8, 128 << 20
    good, bad = LoopbackDatanode(), LoopbackDatanode()
    try:
        datas = [splitmix_bytes(bs, 9000 + i) for i in range(nblk)]
        crcs = [oracle_compute(d, BPC) for d in datas]
        corrupt = datas[5].copy()
        corrupt[77 * BPC + 3] ^= 0x10
        for i in range(nblk):
            good.add_block(900 + i, datas[i], crcs[i], BPC)
            bad.add_block(900 + i, corrupt if i == 5 else datas[i], crcs[i], BPC)
        blocks = [(900 + i, bs) for i in range(nblk)]
        from libhdfs3_amd.engine import InputStream
        replicas = [("127.0.0.1", bad.port), ("127.0.0.1", good.port)]
        with InputStream([(bid, n, replicas) for bid, n in blocks]) as s:
            out = np.empty(4 << 20, np.uint8)
            pos = 0
            for i in range(nblk):
                off = 0
                while off < bs:
                    n = s.read_into(out, 0, min(out.nbytes, bs - off))
                    assert n > 0
                    assert np.array_equal(out[:n], datas[i][off:off + n]), (i, off)
                    off += n
                pos += bs
            assert s.read_into(out) == 0 and s.tell() == nblk * bs == 1 << 30
            st = s.stats()
            assert st["failovers"] == 1 and st["readers_opened"] >= nblk + 1
    finally:
        good.stop()
        bad.stop()
