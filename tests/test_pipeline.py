"""Write-side transport (hdfs3_pipeline, include/hdfs3_client.h): PipelineImpl's OP_WRITE_BLOCK
setup, packet send and ack processing (src/client/Pipeline.cpp:529-841) against loopback
datanodes chained into a real pipeline (first node mirrors to the next; the last one verifies
every CRC word with its own CPU CRC32C, as HDFS's BlockReceiver does).

CPU tests feed the pipeline packets built by the reference restatement (tests/writer_model.py,
CRC words from the oracle): they need no GPU. GPU tests run hdfsWrite -> GPU CRCs -> pipeline
-> datanodes -> hdfsRead (GPU verify) round trips, and compare the words every replica stored
with the oracle."""
import ctypes

import numpy as np
import pytest

from loopback import LoopbackDatanode
from util import oracle_compute, oracle_crc, splitmix_bytes
from writer_model import OutputStreamModel

HOST = "127.0.0.1"


def crc(b: bytes) -> int:
    return oracle_crc(np.frombuffer(b, np.uint8)) if b else 0


@pytest.fixture
def nodes():
    dns = [LoopbackDatanode() for _ in range(3)]
    yield dns
    for d in dns:
        d.stop()


def send_model_packets(pipe, packets):
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


def model_run(data: np.ndarray, ops, bpc=512, packet_size=65536, block_size=1 << 20):
    m = OutputStreamModel(crc, bpc=bpc, packet_size=packet_size, block_size=block_size)
    pos = 0
    for op, n in ops:
        if op == "w":
            m.write(data[pos:pos + n].tobytes())
            pos += n
        elif op == "f":
            m.flush()
        else:
            m.sync()
    m.close()
    return m.sent


def test_three_node_pipeline_stores_every_replica(nodes):
    """2.5 blocks through a 3-node pipeline: every node finalizes every block with the exact
    bytes and the oracle's CRC words; bytesAcked per block = the block's length."""
    from libhdfs3_amd.engine import Pipeline

    bs = 1 << 20
    data = splitmix_bytes(2 * bs + 300_001, 11)
    sent = model_run(data, [("w", 700_000), ("f", 0), ("w", 900_000), ("s", 0), ("w", data.size - 1_600_000)],
                     block_size=bs)
    chain = [(HOST, d.port) for d in nodes]
    blocks = [(9000 + i, chain) for i in range(3)]
    with Pipeline(blocks) as pipe:
        assert send_model_packets(pipe, sent) == 0, pipe.error
        st = pipe.stats()
    assert st["block_bytes_acked"] == [bs, bs, data.size - 2 * bs]
    assert st["acks"] == st["packets"] == len(sent)
    for d in nodes:
        assert d.wait_finalized(3) == 3
        for i in range(3):
            got, words, bpc = d.get_block(9000 + i)
            want = data[i * bs:(i + 1) * bs]
            assert bpc == 512 and np.array_equal(got, want)
            assert np.array_equal(words, oracle_compute(want, 512))
        assert d.write_stats()["checksum_errors"] == 0


def test_flush_waits_for_every_ack(nodes):
    """PipelineImpl::flush = waitForAcks(true): after it returns nothing is outstanding."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import Pipeline

    data = splitmix_bytes(300_000, 3)
    sent = model_run(data, [("w", 300_000), ("f", 0)], block_size=1 << 20)
    flushed = [p for p in sent if not p[1]["last"]]
    with Pipeline([(77, [(HOST, nodes[0].port), (HOST, nodes[1].port)])]) as pipe:
        assert send_model_packets(pipe, flushed) == 0
        assert _native.lib().hdfs3_pipeline_flush(pipe.p) == 0
        assert pipe.stats()["acks"] == len(flushed)


def test_refused_setup_reports_first_bad_link(nodes):
    """createBlockOutputStream (:561-575): a non-SUCCESS connect ack fails with the
    firstBadLink the datanode names — here the second node of the pipeline."""
    from libhdfs3_amd.engine import Pipeline

    nodes[1].set_write_fault(LoopbackDatanode.FAULT_REFUSE_SETUP)
    sent = model_run(splitmix_bytes(5000, 1), [("w", 5000)])
    with Pipeline([(5, [(HOST, d.port) for d in nodes])]) as pipe:
        assert send_model_packets(pipe, sent) == -5  # -EIO
        assert f"Bad connect ack with firstBadLink as 127.0.0.1:{nodes[1].port}" in pipe.error


@pytest.mark.parametrize("bad_node", [0, 2])
def test_ack_error_names_the_node(nodes, bad_node):
    """processAck (:709-720): the last non-SUCCESS reply names the failing node."""
    from libhdfs3_amd.engine import Pipeline

    nodes[bad_node].set_write_fault(LoopbackDatanode.FAULT_ACK_ERROR, 3)
    sent = model_run(splitmix_bytes(600_000, 2), [("w", 600_000)])
    with Pipeline([(6, [(HOST, d.port) for d in nodes])]) as pipe:
        assert send_model_packets(pipe, sent) == -5
        assert f"ack report error at node: 127.0.0.1:{nodes[bad_node].port}" in pipe.error
    for d in nodes:
        assert d.get_block(6) is None  # never finalized


def test_corruption_in_transit_is_caught_by_the_last_node(nodes):
    """A bit flipped on the wire into node 1 is mirrored to node 2, whose CRC check reports
    DT_PROTO_ERROR_CHECKSUM; the client names node 2 and the block is never finalized."""
    from libhdfs3_amd.engine import Pipeline

    nodes[1].set_write_fault(LoopbackDatanode.FAULT_CORRUPT_IN_TRANSIT, 2)
    sent = model_run(splitmix_bytes(400_000, 4), [("w", 400_000)])
    with Pipeline([(8, [(HOST, d.port) for d in nodes])]) as pipe:
        assert send_model_packets(pipe, sent) == -5
        assert f"ack report error at node: 127.0.0.1:{nodes[2].port}" in pipe.error
    assert nodes[2].write_stats()["checksum_errors"] == 1
    assert all(d.get_block(8) is None for d in nodes)


def test_bad_crc_from_the_client_is_rejected(nodes):
    """A packet whose CRC word is wrong (the sender's engine failed) is refused by the last
    node: ERROR_CHECKSUM, surfaced as -EIO."""
    from libhdfs3_amd.engine import Pipeline

    sent = model_run(splitmix_bytes(200_000, 5), [("w", 200_000)])
    buf, info = sent[1]
    bad = bytearray(buf)
    bad[31 + 4 * 7] ^= 0x01  # chunk 7's BE word
    sent[1] = (bytes(bad), info)
    with Pipeline([(10, [(HOST, nodes[0].port)])]) as pipe:
        assert send_model_packets(pipe, sent) == -5
        assert "ack report error at node" in pipe.error


def test_dropped_connection_fails_the_stream(nodes):
    from libhdfs3_amd.engine import Pipeline

    nodes[0].set_write_fault(LoopbackDatanode.FAULT_DROP_AT, 1)
    sent = model_run(splitmix_bytes(300_000, 6), [("w", 300_000)])
    with Pipeline([(12, [(HOST, nodes[0].port)])], timeout_ms=5000) as pipe:
        assert send_model_packets(pipe, sent) == -5
        assert pipe.error


def test_unallocated_block_is_an_error(nodes):
    from libhdfs3_amd.engine import Pipeline

    bs = 1 << 20
    sent = model_run(splitmix_bytes(bs + 10, 7), [("w", bs + 10)], block_size=bs)
    with Pipeline([(13, [(HOST, nodes[0].port)])]) as pipe:
        assert send_model_packets(pipe, sent) == -5
        assert "no block allocated for block 1" in pipe.error


def test_max_unacked_bounds_outstanding_packets(nodes):
    """waitForAcks(false) (:631-633): with max_unacked=2 the writer never gets ahead of the
    acks by more than two packets, and everything still lands."""
    from libhdfs3_amd.engine import Pipeline

    data = splitmix_bytes(1 << 20, 8)
    sent = model_run(data, [("w", 1 << 20)], block_size=1 << 20)
    with Pipeline([(14, [(HOST, d.port) for d in nodes])], max_unacked=2) as pipe:
        assert send_model_packets(pipe, sent) == 0, pipe.error
    for d in nodes:
        assert d.wait_finalized(1) == 1
        assert np.array_equal(d.get_block(14)[0], data)


# ---- GPU: hdfsWrite -> GPU CRCs -> pipeline -> datanodes -> hdfsRead -------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("bpc", [512, 4096])
def test_gpu_write_pipeline_read_round_trip(nodes, bpc):
    """OutputStream(pipeline=...) over a 3-node pipeline with flushes and syncs: every
    replica stores the bytes and exactly the oracle's CRC words, and an InputStream reads the
    file back through GPU verification from any replica."""
    from libhdfs3_amd.engine import InputStream, OutputStream, Pipeline

    bs = 2 << 20
    data = splitmix_bytes(2 * bs + 123_457, 21 + bpc)
    chain = [(HOST, d.port) for d in nodes]
    with Pipeline([(100 + i, chain) for i in range(3)], bytes_per_checksum=bpc) as pipe:
        with OutputStream(pipeline=pipe, bytes_per_checksum=bpc, block_size=bs) as out:
            pos = 0
            for i, n in enumerate([1, 700_000, 511, 65_536 * 3 + 7, 1 << 20, 2 * bs]):
                n = min(n, data.size - pos)
                assert out.write(data[pos:pos + n]) == n
                pos += n
                (out.flush if i % 2 else out.sync)()
                assert pipe.stats()["acks"] == pipe.stats()["packets"]  # flush waited for acks
            if pos < data.size:
                out.write(data[pos:])
        assert pipe.stats()["block_bytes_acked"] == [bs, bs, data.size - 2 * bs]
    for d in nodes:
        assert d.wait_finalized(3) == 3
        for i in range(3):
            got, words, got_bpc = d.get_block(100 + i)
            want = data[i * bs:(i + 1) * bs]
            assert got_bpc == bpc and np.array_equal(got, want)
            assert np.array_equal(words, oracle_compute(want, bpc))
    sizes = [bs, bs, data.size - 2 * bs]
    for d in (nodes[2], nodes[0]):
        with InputStream([(100 + i, sizes[i], [(HOST, d.port)]) for i in range(3)]) as s:
            assert np.array_equal(s.read_fully(data.size), data)


@pytest.mark.gpu
def test_gpu_write_pipeline_failure_is_sticky(nodes):
    """An ack error mid-file fails hdfsWrite/hdfsFlush with EIO and the reference's message,
    and every later call fails the same way (OutputStreamImpl::checkStatus)."""
    import errno

    from libhdfs3_amd.engine import HdfsIOError, OutputStream, Pipeline

    nodes[1].set_write_fault(LoopbackDatanode.FAULT_ACK_ERROR, 5)
    data = splitmix_bytes(4 << 20, 33)
    with Pipeline([(200, [(HOST, d.port) for d in nodes])]) as pipe:
        out = OutputStream(pipeline=pipe, block_size=8 << 20, batch_packets=4)
        with pytest.raises(HdfsIOError) as e:
            out.write(data)
            out.flush()
        assert e.value.errno == errno.EIO and "ack report error at node" in str(e.value)
        with pytest.raises(HdfsIOError):
            out.write(data[:10])
        with pytest.raises(HdfsIOError):
            out.close()
