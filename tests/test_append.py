"""Append to an existing file (row a9 of SURVEY.md §8): OutputStreamImpl::initAppend
(src/client/OutputStreamImpl.cpp:172-230, 332-337) and PipelineImpl(append = true)
(src/client/Pipeline.cpp:58-81, 214-335, 529-549).

The file's last block lives on loopback datanodes (tools/loopback). An append opens a
PIPELINE_SETUP_APPEND pipeline to that block's replicas (minBytesRcvd = its length, the new
generation stamp), sends a first packet of ONE chunk that fills up the partial chunk (its CRC over
the new bytes only; the datanode recomputes the stored word of the whole chunk), then packets of the
configured size; further blocks go through PIPELINE_SETUP_CREATE.

CPU tests drive the pipeline with packets from the reference restatement (tests/writer_model.py,
CRC words from the oracle). GPU tests run the product write path (GPU CRCs) through hdfs3_output_*
and through hdfsOpenFile(O_WRONLY | O_APPEND) / hdfsWrite / hdfsCloseFile, and read the whole file
back with hdfsRead (GPU verify). Packet framing is pinned by the model only (parity unpinned by the
reference: it has no packet test); the stored words and bytes are pinned by the oracle."""
import ctypes
import os

import numpy as np
import pytest

from loopback import LoopbackDatanode
from util import oracle_compute, oracle_crc, splitmix_bytes
from writer_model import OutputStreamModel

HOST = "127.0.0.1"
BS = 1 << 20
POOL = b"BP-loopback"


def crc(b: bytes) -> int:
    return oracle_crc(np.frombuffer(b, np.uint8)) if b else 0


@pytest.fixture
def nodes():
    dns = [LoopbackDatanode() for _ in range(3)]
    yield dns
    for d in dns:
        d.stop()


def existing_file(nodes, length, first_id, seed, bpc=512):
    """A file of `length` bytes stored on every node (blocks first_id, first_id + 1, ...):
    [(block_id, num_bytes)] and the bytes."""
    data = splitmix_bytes(length, seed)
    blocks = []
    for i, off in enumerate(range(0, length, BS)):
        part = np.ascontiguousarray(data[off:off + BS])
        words = oracle_compute(part, bpc)
        for d in nodes:
            d.add_block(first_id + i, part, words, bpc)
        blocks.append((first_id + i, part.size))
    return blocks, data


def model_append_packets(length, last_bytes, payload, ops, bpc=512, packet_size=65536):
    m = OutputStreamModel(crc, bpc=bpc, packet_size=packet_size, block_size=BS, append=(length, last_bytes))
    pos = 0
    for op, n in ops:
        if op == "w":
            m.write(payload[pos:pos + n].tobytes())
            pos += n
        elif op == "f":
            m.flush()
        else:
            m.sync()
    m.close()
    return m.sent


def send(pipe, packets):
    from libhdfs3_amd import _native

    lib = _native.lib()
    for buf, d in packets:
        info = _native.PacketInfo(d["seqno"], d["offset_in_block"], d["block_index"], d["data_len"], d["num_chunks"],
                                  int(d["last"]))
        b = ctypes.create_string_buffer(buf, len(buf))
        rc = lib.hdfs3_pipeline_send(pipe.p, b, len(buf), ctypes.byref(info))
        if rc:
            return rc
    return 0


def check_replicas(nodes, blocks, whole, bpc=512, gs=None):
    """every node holds every block with the file's bytes and the oracle's words over them"""
    off = 0
    for bid, n in blocks:
        want = whole[off:off + n]
        for d in nodes:
            assert d.wait_finalized(0) >= 0
            got = d.get_block(bid)
            assert got is not None, (bid, d.port)
            data, words, got_bpc = got
            assert got_bpc == bpc and np.array_equal(data, want), (bid, d.port)
            assert np.array_equal(words, oracle_compute(want, bpc)), (bid, d.port)
            if gs is not None and bid in gs:
                assert d.block_gs(bid) == gs[bid]
        off += n
    assert off == whole.size


@pytest.mark.parametrize("tail", [100, 511, 1, 0, BS - 512, BS - 1])
def test_model_packets_append_through_loopback_pipeline(nodes, tail):
    """CPU: the reference model's append packets through hdfs3_pipeline_open_append. The last
    block (tail bytes; 0 = the file ends on a chunk boundary 7 chunks in) grows on every replica,
    the chunk the append completed gets its word recomputed over the whole chunk, the block takes
    the new generation stamp, and the bytes beyond it go to a new block."""
    from libhdfs3_amd.engine import Pipeline

    tail = tail or 7 * 512
    length = 2 * BS + tail
    blocks, old = existing_file(nodes, length, 500, seed=tail % 1000 + 1)
    payload = splitmix_bytes(BS + 12345, 77)
    ops = [("w", 10), ("f", 0), ("w", 70_000), ("s", 0), ("w", payload.size - 70_010)]
    sent = model_append_packets(length, tail, payload, ops)
    assert sent[0][1]["offset_in_block"] == tail
    chain = [(HOST, d.port) for d in nodes]
    with Pipeline([(502, chain), (503, chain), (504, chain)], append=(tail, 9), generation_stamp=1) as pipe:
        assert send(pipe, sent) == 0, pipe.error
        acked = pipe.stats()["block_bytes_acked"]
        assert pipe.generation_stamp(0) == 9 and pipe.generation_stamp(1) == 1
    whole = np.concatenate([old, payload])
    sizes = [BS] * (whole.size // BS) + [whole.size % BS]
    assert acked == sizes[2:] + [0] * (5 - len(sizes))
    for d in nodes:
        assert d.wait_finalized(len(sizes) - 2) == len(sizes) - 2
    check_replicas(nodes, [(500 + i, n) for i, n in enumerate(sizes)], whole, gs={502: 9})


def test_append_setup_refused_on_length_mismatch(nodes):
    """minBytesRcvd must match the replica: a stale length is refused at setup (Bad connect ack)."""
    from libhdfs3_amd.engine import Pipeline

    blocks, _ = existing_file(nodes[:1], 1000, 600, seed=3)
    sent = model_append_packets(1000, 999, splitmix_bytes(100, 4), [("w", 100)])
    with Pipeline([(600, [(HOST, nodes[0].port)])], append=(999, 2)) as pipe:
        assert send(pipe, sent) == -5  # -EIO
        assert "Bad connect ack" in pipe.error
    assert nodes[0].get_block(600)[0].size == 1000  # untouched


def test_append_requires_a_newer_generation_stamp():
    from libhdfs3_amd.engine import Pipeline
    from libhdfs3_amd._native import Hdfs3CrcError

    with pytest.raises(Hdfs3CrcError):
        Pipeline([(1, [(HOST, 1)])], append=(10, 1), generation_stamp=1)


# ---- GPU: the product write path ---------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("tail", [100, 7 * 512, BS - 512])
def test_gpu_append_stream_then_read_whole_file(nodes, tail):
    """hdfs3_output_open_pipeline_append over the append pipeline: GPU CRCs, packets as the model,
    every replica holds old + new bytes with the oracle's words, and hdfsRead (hdfs3_input_*, GPU
    verify) returns the whole file from any replica."""
    from libhdfs3_amd.engine import InputStream, OutputStream, Pipeline

    length = BS + tail
    blocks, old = existing_file(nodes, length, 700, seed=tail % 997 + 5)
    payload = splitmix_bytes(2 * BS + 4321, 78)
    chain = [(HOST, d.port) for d in nodes]
    with Pipeline([(701 + i, chain) for i in range(4)], append=(tail, 5)) as pipe:
        with OutputStream(pipeline=pipe, append=(length, tail), block_size=BS, batch_packets=8) as out:
            assert out.tell() == length
            pos = 0
            for n in (7, 1000, 100_000, 512, 1 << 20, payload.size):
                n = min(n, payload.size - pos)
                if n <= 0:
                    break
                assert out.write(payload[pos:pos + n]) == n
                pos += n
                out.flush()
            assert out.tell() == length + payload.size
    whole = np.concatenate([old, payload])
    sizes = [BS] * (whole.size // BS) + ([whole.size % BS] if whole.size % BS else [])
    for d in nodes:
        assert d.wait_finalized(len(sizes) - 1) >= len(sizes) - 1
    check_replicas(nodes, [(700 + i, n) for i, n in enumerate(sizes)], whole, gs={701: 5})
    for d in (nodes[0], nodes[2]):
        with InputStream([(700 + i, n, [(HOST, d.port)]) for i, n in enumerate(sizes)]) as s:
            assert np.array_equal(s.read_fully(whole.size), whole)


class Hdfs:
    """hdfs.h through ctypes (include/hdfs3_hdfs.h) over an hdfs3_fs_new table."""

    def __init__(self, block_size=BS):
        from libhdfs3_amd import _native

        self.lib = _native.lib()
        self._native = _native
        wopts = _native.WriterOpts(0, 512, 65536, block_size, 8)
        self.fs = self.lib.hdfs3_fs_new(b"append-test", None, ctypes.byref(wopts))
        assert self.fs
        self._keep = []

    def located(self, blocks, gs=1):
        from libhdfs3_amd.engine import _located_blocks

        arr, keep = _located_blocks(blocks, POOL, gs)
        self._keep.append(keep)
        return arr

    def add_file(self, path, blocks, gs=1):
        assert self.lib.hdfs3_fs_add_file(self.fs, path, self.located(blocks, gs), len(blocks)) == 0

    def set_pipeline(self, path, blocks):
        arr = self.located([(bid, 0, nodes) for bid, nodes in blocks])
        assert self.lib.hdfs3_fs_set_pipeline(self.fs, path, arr, len(blocks)) == 0

    def write_file(self, path, flags, pieces):
        f = self.lib.hdfsOpenFile(self.fs, path, flags, 0, 0, 0)
        assert f, (ctypes.get_errno(), self.lib.hdfsGetLastError())
        tell0 = self.lib.hdfsTell(self.fs, f)
        for p in pieces:
            buf = np.ascontiguousarray(p)
            assert self.lib.hdfsWrite(self.fs, f, buf.ctypes.data, buf.nbytes) == buf.nbytes
            assert self.lib.hdfsHFlush(self.fs, f) == 0
        assert self.lib.hdfsCloseFile(self.fs, f) == 0, self.lib.hdfsGetLastError()
        return tell0

    def read_file(self, path, n):
        f = self.lib.hdfsOpenFile(self.fs, path, os.O_RDONLY, 0, 0, 0)
        assert f, self.lib.hdfsGetLastError()
        out = np.zeros(n + 1, np.uint8)
        got = 0
        while True:
            r = self.lib.hdfsRead(self.fs, f, out.ctypes.data + got, min(1 << 20, out.nbytes - got))
            assert r >= 0, self.lib.hdfsGetLastError()
            if r == 0:
                break
            got += r
        assert self.lib.hdfsCloseFile(self.fs, f) == 0
        return out[:got]

    def close(self):
        self.lib.hdfsDisconnect(self.fs)


@pytest.mark.gpu
@pytest.mark.parametrize("tail", [300, 0, BS - 512])
def test_gpu_hdfs_open_append_then_hdfsRead(nodes, tail):
    """hdfsOpenFile(O_WRONLY | O_APPEND): a file written with hdfsWrite through a 3-node pipeline
    (tail bytes into its last block; 0 = ends on a block boundary) is appended to twice through
    hdfs.h, each append closed cleanly; hdfsRead then returns the whole file and the appended block
    carries the stamp registered with hdfs3_fs_set_append_stamp."""
    h = Hdfs()
    try:
        chain = [(HOST, d.port) for d in nodes]
        path = b"/append/f"
        first = splitmix_bytes(BS + tail, 90 + tail % 7)
        h.set_pipeline(path, [(800 + i, chain) for i in range(2)])
        h.write_file(path, os.O_WRONLY | os.O_CREAT, [first])
        a1, a2 = splitmix_bytes(777, 91), splitmix_bytes(BS + 5000, 92)
        # the first append continues block 801 (or starts one when the file ended on a block
        # boundary); blocks beyond come from the registered pipeline
        h.set_pipeline(path, [(810 + i, chain) for i in range(3)])
        assert h.lib.hdfs3_fs_set_append_stamp(h.fs, path, 40) == 0
        assert h.write_file(path, os.O_WRONLY | os.O_APPEND, [a1[:5], a1[5:]]) == first.size
        assert np.array_equal(h.read_file(path, first.size + a1.size), np.concatenate([first, a1]))
        assert h.lib.hdfs3_fs_set_append_stamp(h.fs, path, 41) == 0
        h.set_pipeline(path, [(820 + i, chain) for i in range(3)])
        assert h.write_file(path, os.O_WRONLY | os.O_APPEND, [a2]) == first.size + a1.size
        whole = np.concatenate([first, a1, a2])
        assert np.array_equal(h.read_file(path, whole.size), whole)
        if tail == 300:
            assert all(d.block_gs(801) == 41 for d in nodes)  # appended to twice
    finally:
        h.close()


@pytest.mark.gpu
def test_gpu_hdfs_append_missing_file_is_enoent():
    import errno

    h = Hdfs()
    try:
        f = h.lib.hdfsOpenFile(h.fs, b"/nope", os.O_WRONLY | os.O_APPEND, 0, 0, 0)
        assert not f and ctypes.get_errno() == errno.ENOENT
    finally:
        h.close()


@pytest.mark.gpu
def test_gpu_hdfs_append_block_size_must_match_the_file(nodes):
    """the block size an append uses is the file's (FileStatus::getBlockSize in
    OutputStreamImpl.cpp:196-230). A caller's size that disagrees with a file of two or more
    blocks, or a file whose only block is larger than the stream's block size, is refused with
    EINVAL before anything is written (the copy length into the packet arena used to wrap); a
    filesystem whose default block size differs from the file's appends with the file's."""
    import errno

    chain = [(HOST, d.port) for d in nodes]
    blocks, data = existing_file(nodes, 2 * BS + 700, 900, 21)
    h = Hdfs(block_size=BS // 2)  # the fs default disagrees with the file's BS
    try:
        path = b"/append/bs"
        h.add_file(path, [(bid, n, chain) for bid, n in blocks])
        f = h.lib.hdfsOpenFile(h.fs, path, os.O_WRONLY | os.O_APPEND, 0, 0, 2 * BS)
        assert not f and ctypes.get_errno() == errno.EINVAL
        extra = splitmix_bytes(5000, 22)
        assert h.write_file(path, os.O_WRONLY | os.O_APPEND, [extra]) == data.size  # the file's BS
        whole = np.concatenate([data, extra])
        assert np.array_equal(h.read_file(path, whole.size), whole)
        # one block bigger than the stream's block size: refused, nothing sent
        one, _ = existing_file(nodes, BS - 100, 950, 23)
        h2 = Hdfs(block_size=BS // 4)
        try:
            h2.add_file(b"/append/one", [(bid, n, chain) for bid, n in one])
            f = h2.lib.hdfsOpenFile(h2.fs, b"/append/one", os.O_WRONLY | os.O_APPEND, 0, 0, 0)
            assert not f and ctypes.get_errno() == errno.EINVAL
        finally:
            h2.close()
    finally:
        h.close()


@pytest.mark.gpu
def test_gpu_output_open_append_rejects_last_block_beyond_block_size():
    """hdfs3_output_open_append: last_block_bytes must be < block_size and agree with
    file_length mod block_size (-EINVAL otherwise), so a block's remaining room is never negative.
    A file that ends on a block boundary keeps the reference's "last block is full" EIO first
    (OutputStreamImpl.cpp:192-199; test_output_stream.py::test_append_to_full_last_block_is_eio)."""
    import errno

    from libhdfs3_amd import _native

    lib = _native.lib()
    opts = _native.WriterOpts(0, 512, 65536, BS, 8)
    sink = _native.PACKET_SINK(lambda u, p, n, i: 0)
    for file_length, last in ((3 * BS + 10, BS + 10), (BS + 10, 30), (5 * BS + 7, 2 * BS + 7)):
        ai = _native.AppendInfo(file_length, last)
        out = ctypes.c_void_p()
        rc = lib.hdfs3_output_open_append(ctypes.byref(opts), ctypes.byref(ai), sink, None, ctypes.byref(out))
        assert rc == -errno.EINVAL, (file_length, last, rc)
        assert not out.value


@pytest.mark.gpu
def test_gpu_hdfs_second_append_without_new_stamp_or_pipeline(nodes):
    """ADVICE r3 (medium/low): a write consumes the pipeline table and the append stamp it used.
    A second append that registers neither continues the last block with the last stamp + 1 and
    no block id is reused; a stale table naming one of the file's blocks is refused."""
    import errno

    h = Hdfs()
    try:
        chain = [(HOST, d.port) for d in nodes]
        path = b"/append/twice"
        first = splitmix_bytes(BS + 300, 31)
        h.set_pipeline(path, [(830 + i, chain) for i in range(2)])
        h.write_file(path, os.O_WRONLY | os.O_CREAT, [first])
        a1, a2 = splitmix_bytes(900, 32), splitmix_bytes(1500, 33)
        assert h.lib.hdfs3_fs_set_append_stamp(h.fs, path, 40) == 0
        assert h.write_file(path, os.O_WRONLY | os.O_APPEND, [a1]) == first.size
        # neither a stamp nor a pipeline registered: the last block, stamp 41
        assert h.write_file(path, os.O_WRONLY | os.O_APPEND, [a2]) == first.size + a1.size
        assert all(d.block_gs(831) == 41 for d in nodes)
        whole = np.concatenate([first, a1, a2])
        assert np.array_equal(h.read_file(path, whole.size), whole)
        # a table naming the file's own block 831 is an addBlock that cannot happen
        h.set_pipeline(path, [(831, chain)])
        f = h.lib.hdfsOpenFile(h.fs, path, os.O_WRONLY | os.O_APPEND, 0, 0, 0)
        assert not f and ctypes.get_errno() == errno.EINVAL
    finally:
        h.close()


@pytest.mark.gpu
def test_gpu_hdfs_append_one_block_file_uses_its_own_block_size(nodes):
    """FileStatus::getBlockSize decides where an append continues
    (OutputStreamImpl.cpp:196-230). A one-block file written with a 512 KiB block size (the session's
    is 1 MiB) that filled its block: a clean close records its block size, so the append opens a new
    block (the registered pipeline's) instead of continuing the full block past 512 KiB; a caller
    size that disagrees is refused; hdfs3_fs_set_block_size states it for a registered file."""
    import errno

    h = Hdfs()
    try:
        chain = [(HOST, d.port) for d in nodes]
        path = b"/append/one-block"
        half = BS // 2
        first = splitmix_bytes(half, 61)
        h.set_pipeline(path, [(870, chain)])
        f = h.lib.hdfsOpenFile(h.fs, path, os.O_WRONLY | os.O_CREAT, 0, 0, half)
        assert f, h.lib.hdfsGetLastError()
        assert h.lib.hdfsWrite(h.fs, f, first.ctypes.data, first.nbytes) == first.nbytes
        assert h.lib.hdfsCloseFile(h.fs, f) == 0, h.lib.hdfsGetLastError()
        # the caller's 1 MiB disagrees with the file's 512 KiB
        h.set_pipeline(path, [(871, chain)])
        f = h.lib.hdfsOpenFile(h.fs, path, os.O_WRONLY | os.O_APPEND, 0, 0, BS)
        assert not f and ctypes.get_errno() == errno.EINVAL
        more = splitmix_bytes(1000, 62)
        assert h.write_file(path, os.O_WRONLY | os.O_APPEND, [more]) == first.size
        assert all(d.get_block(870)[0].size == half for d in nodes)  # the full block stays full
        got = nodes[-1].get_block(871)
        assert got is not None and np.array_equal(got[0], more)
        assert np.array_equal(h.read_file(path, half + more.size), np.concatenate([first, more]))
        # a registered (not written) one-block file: its block size comes from hdfs3_fs_set_block_size
        path2 = b"/append/registered"
        assert h.lib.hdfs3_fs_set_block_size(h.fs, path2, 0) == -1 and ctypes.get_errno() == errno.EINVAL
        h.add_file(path2, [(870, half, chain)])
        assert h.lib.hdfs3_fs_set_block_size(h.fs, path2, half) == 0
        f = h.lib.hdfsOpenFile(h.fs, path2, os.O_WRONLY | os.O_APPEND, 0, 0, BS)
        assert not f and ctypes.get_errno() == errno.EINVAL
    finally:
        h.close()


@pytest.mark.gpu
def test_gpu_hdfs_append_guessed_block_size_is_not_recorded(nodes):
    """an append to a one-block file of unknown block size only guesses the size (the
    caller's, else the session's). A clean close must not record that guess as the file's FileStatus
    block size: a later append with another caller size is not refused for "block size differs", and
    appends with that caller's size."""
    h = Hdfs()
    try:
        chain = [(HOST, d.port) for d in nodes]
        path = b"/append/guess"
        one, data = existing_file(nodes, 3000, 990, 71)
        h.add_file(path, [(bid, n, chain) for bid, n in one])
        a1, a2 = splitmix_bytes(700, 72), splitmix_bytes(900, 73)
        assert h.lib.hdfs3_fs_set_append_stamp(h.fs, path, 40) == 0
        f = h.lib.hdfsOpenFile(h.fs, path, os.O_WRONLY | os.O_APPEND, 0, 0, BS)  # a guess: 1 MiB
        assert f, h.lib.hdfsGetLastError()
        assert h.lib.hdfsWrite(h.fs, f, a1.ctypes.data, a1.nbytes) == a1.nbytes
        assert h.lib.hdfsCloseFile(h.fs, f) == 0, h.lib.hdfsGetLastError()
        assert h.lib.hdfs3_fs_set_append_stamp(h.fs, path, 41) == 0
        f = h.lib.hdfsOpenFile(h.fs, path, os.O_WRONLY | os.O_APPEND, 0, 0, BS // 2)  # another guess
        assert f, h.lib.hdfsGetLastError()
        assert h.lib.hdfsWrite(h.fs, f, a2.ctypes.data, a2.nbytes) == a2.nbytes
        assert h.lib.hdfsCloseFile(h.fs, f) == 0, h.lib.hdfsGetLastError()
        whole = np.concatenate([data, a1, a2])
        assert np.array_equal(h.read_file(path, whole.size), whole)
    finally:
        h.close()
