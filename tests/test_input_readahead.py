"""GPU tests of the opt-in block read-ahead of hdfs3_input_stream (hdfs3_input_set_readahead).

The reference reads one block at a time (InputStreamImpl::readOneBlock, InputStreamImpl.cpp
:616-712). With read-ahead on, the readers of the blocks after the current one are opened
early, with deep rings, so their receiver threads read and verify ahead; the cursor then
takes each over when it reaches its block. Everything observable through
hdfsRead must stay the reference's: the same bytes, never two blocks in one call, the same
ChecksumException -> next-replica failover, EIO after exactly the verified bytes when every
replica is bad. Each case is compared with the same stream without read-ahead."""
import errno

import numpy as np
import pytest

from util import oracle_compute, splitmix_bytes

pytestmark = pytest.mark.gpu

BPC = 512
SIZES = [2 << 20] * 5 + [700_001]  # six blocks, ragged last block with a short last chunk


@pytest.fixture(scope="module")
def cluster():
    from loopback import LoopbackDatanode

    a, b = LoopbackDatanode(), LoopbackDatanode()
    blocks, parts = [], []
    for i, n in enumerate(SIZES):
        d = splitmix_bytes(n, 900 + i)
        c = oracle_compute(d, BPC)
        for node in (a, b):
            node.add_block(900 + i, d, c, BPC)
        blocks.append((900 + i, n))
        parts.append(d)
    yield a, b, blocks, np.concatenate(parts)
    a.stop()
    b.stop()


def _stream(blocks, replicas, ahead=0, cap=0, **kw):
    from libhdfs3_amd.engine import InputStream

    s = InputStream([(bid, n, replicas) for bid, n in blocks], **kw)
    if ahead:
        s.set_readahead(ahead, cap)
    return s


def _read_all(s, total, piece=768 * 1024):
    """hdfsRead loop; returns (bytes, per-call (pos, n)) and checks no call crosses a block."""
    out = np.empty(total, np.uint8)
    starts = np.cumsum([0] + SIZES)
    pos, calls = 0, []
    while pos < total:
        n = s.read_into(out, pos, min(piece, total - pos))
        if n == 0:
            break
        blk = np.searchsorted(starts, pos, side="right") - 1
        assert pos + n <= starts[blk + 1]  # readOneBlock: never two blocks in one call
        calls.append((pos, n))
        pos += n
    return out[:pos], calls


@pytest.mark.parametrize("ahead,cap", [(1, 0), (2, 0), (8, 0), (2, 1 << 20), (3, 300_000)])
def test_sequential_read_equals_file(cluster, ahead, cap):
    a, b, blocks, whole = cluster
    with _stream(blocks, [("127.0.0.1", a.port)], ahead, cap) as s:
        got, _ = _read_all(s, whole.nbytes)
        assert np.array_equal(got, whole)
        assert s.read_into(np.zeros(8, np.uint8)) == 0
        st = s.stats()
        assert st["failovers"] == 0
        # block 0 on demand, every later block through a reader opened ahead of the cursor (a
        # cap only makes its ring shallower: it still streams the whole block)
        assert st["prefetch_readers_opened"] == len(SIZES) - 1
        assert st["readers_opened"] == 1


def test_corrupt_prefetched_replica_fails_over(cluster):
    from loopback import LoopbackDatanode

    a, b, blocks, whole = cluster
    bad = LoopbackDatanode()
    try:
        off = 0
        for i, (bid, n) in enumerate(blocks):
            d = whole[off:off + n].copy()
            c = oracle_compute(d, BPC)
            if i in (2, 4):
                d[n // 2 + 123] ^= 0x08  # corrupt replica of two prefetched blocks
            bad.add_block(bid, d, c, BPC)
            off += n
        reps = [("127.0.0.1", bad.port), ("127.0.0.1", b.port)]
        for ahead in (0, 2):
            with _stream(blocks, reps, ahead) as s:
                got, _ = _read_all(s, whole.nbytes)
                assert np.array_equal(got, whole), ahead
                assert s.stats()["failovers"] == 2, ahead
    finally:
        bad.stop()


def test_every_replica_bad_eio_after_the_same_bytes(cluster):
    from libhdfs3_amd.engine import HdfsIOError
    from loopback import LoopbackDatanode

    a, b, blocks, whole = cluster
    bad = LoopbackDatanode()
    try:
        off = 0
        for i, (bid, n) in enumerate(blocks):
            d = whole[off:off + n].copy()
            c = oracle_compute(d, BPC)
            if i == 3:
                d[1_000_000] ^= 0x01
            bad.add_block(bid, d, c, BPC)
            off += n
        delivered = {}
        for ahead in (0, 1, 3):
            with _stream(blocks, [("127.0.0.1", bad.port)], ahead) as s:
                out = np.zeros(whole.nbytes, np.uint8)
                pos = 0
                with pytest.raises(HdfsIOError) as ei:
                    while True:
                        n = s.read_into(out, pos, 1 << 20)
                        assert n > 0
                        pos += n
                assert ei.value.errno == errno.EIO and "all nodes have been tried" in str(ei.value)
                assert np.array_equal(out[:pos], whole[:pos])
                delivered[ahead] = pos
        # the bytes handed out before EIO are the on-demand reader's, read-ahead or not
        assert delivered[1] == delivered[0] == delivered[3]
        assert sum(SIZES[:3]) <= delivered[0] <= sum(SIZES[:3]) + 1_000_000
    finally:
        bad.stop()


def test_dropped_connection_during_prefetch(cluster):
    from loopback import LoopbackDatanode

    a, b, blocks, whole = cluster
    flaky = LoopbackDatanode()
    try:
        off = 0
        for bid, n in blocks:
            d = whole[off:off + n]
            flaky.add_block(bid, d, oracle_compute(d, BPC), BPC)
            off += n
        flaky.set_fail_after(1 << 20)  # every block > 1 MiB is cut after 1 MiB
        with _stream(blocks, [("127.0.0.1", flaky.port), ("127.0.0.1", a.port)], 3, timeout_ms=5000) as s:
            got, _ = _read_all(s, whole.nbytes)
            assert np.array_equal(got, whole)
            assert s.stats()["failovers"] == 5  # blocks 0-4 (the last block is 700 KB)
    finally:
        flaky.stop()


def test_seeks_into_and_out_of_prefetched_blocks(cluster):
    a, b, blocks, whole = cluster
    starts = np.cumsum([0] + SIZES)
    with _stream(blocks, [("127.0.0.1", a.port)], 3) as s:
        buf = np.zeros(4096, np.uint8)
        assert s.read_into(buf) == 4096  # block 0 on demand, blocks 1-3 prefetching
        for pos in [int(starts[2]) + 5, int(starts[2]) + 100, int(starts[1]) + 77, 10, int(starts[5]) + 1,
                    int(starts[3]) - 3, whole.nbytes - 9]:
            s.seek(pos)
            n = s.read_into(buf, 0, 4096)
            assert n > 0 and np.array_equal(buf[:n], whole[pos:pos + n]), pos
        s.seek(int(starts[1]))
        got, _ = _read_all(s, whole.nbytes - int(starts[1]))
        assert np.array_equal(got, whole[int(starts[1]):])


def test_close_with_prefetches_in_flight(cluster):
    a, b, blocks, whole = cluster
    for _ in range(5):
        with _stream(blocks, [("127.0.0.1", a.port)], 4) as s:
            buf = np.zeros(10, np.uint8)
            assert s.read_into(buf) == 10 and np.array_equal(buf, whole[:10])
        # closing joins the prefetch threads; the next stream starts clean


def test_readahead_off_again_and_pread_unaffected(cluster):
    a, b, blocks, whole = cluster
    with _stream(blocks, [("127.0.0.1", a.port)], 2) as s:
        first = np.zeros(SIZES[0], np.uint8)
        assert s.read_into(first) == SIZES[0] and np.array_equal(first, whole[:SIZES[0]])
        s.set_readahead(0)
        out = np.zeros(1 << 20, np.uint8)
        pos = SIZES[0] + SIZES[1] - 1000
        assert s.pread_into(pos, out) == out.nbytes and np.array_equal(out, whole[pos:pos + out.nbytes])
        got, _ = _read_all(s, whole.nbytes - SIZES[0])
        assert np.array_equal(got, whole[SIZES[0]:])


@pytest.mark.parametrize("ahead", [0, 2, 5])
def test_random_walk_of_reads_seeks_and_preads(cluster, ahead):
    """A seeded random walk of hdfsRead (1 B to 3 MiB), hdfsSeek (anywhere, block starts
    included) and hdfsPread over the 6-block file, with and without read-ahead: every byte
    equals the file's, read never crosses a block, tell follows the cursor."""
    a, b, blocks, whole = cluster
    starts = np.cumsum([0] + SIZES)
    rng = np.random.default_rng(ahead + 77)
    with _stream(blocks, [("127.0.0.1", a.port)], ahead) as s:
        pos = 0
        for _ in range(80):
            op = rng.integers(0, 10)
            if op < 6:
                n = int(rng.integers(1, 3 << 20))
                buf = np.zeros(n, np.uint8)
                got = s.read_into(buf)
                if pos >= whole.nbytes:
                    assert got == 0
                    continue
                blk = np.searchsorted(starts, pos, side="right") - 1
                assert 0 < got <= n and pos + got <= starts[blk + 1]
                assert np.array_equal(buf[:got], whole[pos:pos + got])
                pos += got
            elif op < 8:
                pos = int(rng.choice([rng.integers(0, whole.nbytes), starts[rng.integers(0, len(SIZES))]]))
                s.seek(pos)
            else:
                p = int(rng.integers(0, whole.nbytes))
                n = int(rng.integers(1, 3 << 20))
                buf = np.zeros(n, np.uint8)
                got = s.pread_into(p, buf)
                assert got == min(n, whole.nbytes - p) and np.array_equal(buf[:got], whole[p:p + got])
            assert s.tell() == pos


def test_local_fault_in_a_prefetched_reader_is_read_on_demand(cluster):
    """A read-ahead reader whose pinned arena cannot be allocated (a local fault, injected through
    the measurement library's hook) is dropped and its block read again on demand on the stream's
    own context: the same bytes as with read-ahead off, no replica failed over, and the fault only
    counted (turning read-ahead on must not make a read fail)."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import InputStream

    a, b, blocks, whole = cluster
    lab = _native.lab()
    try:
        lab.hdfs3x_fail_prefetch_arenas(3)
        with InputStream([(bid, n, [("127.0.0.1", a.port)]) for bid, n in blocks], lib=lab) as s:
            s.set_readahead(2)
            got, _ = _read_all(s, whole.nbytes)
            st = s.stats()
        assert np.array_equal(got, whole)
        assert st["failovers"] == 0 and st["prefetch_local_faults"] >= 1
    finally:
        lab.hdfs3x_fail_prefetch_arenas(0)


def test_readahead_depth_is_bounded(cluster):
    from libhdfs3_amd._native import Hdfs3CrcError

    a, b, blocks, whole = cluster
    with _stream(blocks, [("127.0.0.1", a.port)]) as s:
        s.set_readahead(8)
        with pytest.raises(Hdfs3CrcError):
            s.set_readahead(9)


def test_pool_pinned_memory_stays_under_the_cap(cluster):
    """Streams with deep read-ahead rings opened and closed over many blocks leave at most the
    pool's pinned cap retained (hdfs3_crc_pool_stats_get), and hdfs3_crc_pool_trim empties it."""
    import ctypes

    from libhdfs3_amd import _native

    a, b, blocks, whole = cluster
    lib = _native.lib()
    st = _native.PoolStats()
    for rep in range(3):
        for ahead in (2, 5):
            with _stream(blocks, [("127.0.0.1", a.port)], ahead) as s:
                got, _ = _read_all(s, whole.nbytes)
                assert np.array_equal(got, whole)
            assert lib.hdfs3_crc_pool_stats_get(ctypes.byref(st)) == 0
            assert st.pinned_bytes <= st.pinned_cap_bytes, (st.pinned_bytes, st.pinned_cap_bytes)
    assert st.pinned_cap_bytes == 1 << 30 and st.pooled_contexts > 0
    assert lib.hdfs3_crc_pool_trim() == st.pooled_contexts
    assert lib.hdfs3_crc_pool_stats_get(ctypes.byref(st)) == 0
    assert st.pooled_contexts == 0 and st.pinned_bytes == 0
