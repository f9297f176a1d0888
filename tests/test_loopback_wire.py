"""CPU tests of the data-transfer wire path: the loopback datanode (C++, the product's
wire codec) against an independent Python client (tests/dtp.py). Checks the OP_READ_BLOCK
framing, BlockOpResponseProto/ChecksumProto, packet headers (31 bytes, seqno, offsets,
packetLen = dataLen + CRC bytes + 4), chunk-aligned first packet, the empty last packet,
the final CHECKSUM_OK status, and every CRC word against the oracle."""
import numpy as np
import pytest

from dtp import Conn, packet_header, parse_packet_header
from util import oracle_compute, splitmix_bytes


@pytest.fixture(scope="module")
def datanode():
    from loopback import LoopbackDatanode

    dn = LoopbackDatanode()

    def add(block_id, data, bpc, crc=None, ctype=2):
        crc = oracle_compute(data, bpc) if crc is None else crc
        dn.add_block(block_id, data, crc, bpc, ctype)
        return crc

    yield dn, dn.port, add
    dn.stop()


def test_packet_header_layout_matches_reference_size():
    h = packet_header(4 + 512 + 4, 4096, 3, False, 512)
    assert len(h) == 31  # PacketHeader::GetPkgHeaderSize (PacketHeader.cpp:38-45)
    assert parse_packet_header(h) == {"packet_len": 520, "offset": 4096, "seqno": 3, "last": False,
                                      "data_len": 512}


@pytest.mark.parametrize("bpc", [512, 4096])
def test_full_block_read(datanode, bpc):
    lb, port, add = datanode
    data = splitmix_bytes(1 << 20, bpc)
    crc = add(100 + bpc, data, bpc)
    c = Conn(port)
    resp, packets = c.read_block(100 + bpc, 0, data.nbytes)
    c.send_status(6)
    c.close()
    assert resp[1][0] == 0
    got, words = bytearray(), bytearray()
    for i, (h, cb, d) in enumerate(packets):
        assert h["seqno"] == i
        if h["last"]:
            assert h["data_len"] == 0 and h["packet_len"] == 4 and i == len(packets) - 1
            continue
        assert h["offset"] == len(got)
        assert h["packet_len"] == 4 + h["data_len"] + len(cb)
        got += d
        words += cb
    assert bytes(got) == data.tobytes()
    assert bytes(words) == crc.tobytes()
    # every CRC word as the datanode served it checks out against the oracle
    assert np.array_equal(np.frombuffer(bytes(words), np.uint8), oracle_compute(data, bpc))


def test_ranged_read_aligns_back_to_chunk(datanode):
    lb, port, add = datanode
    data = splitmix_bytes(300_000 + 77, 9)  # short last chunk
    add(7, data, 512)
    c = Conn(port)
    resp, packets = c.read_block(7, 1000, 5000)
    c.send_status(6)
    c.close()
    from dtp import parse
    info = parse(resp[4][0])
    assert info[2][0] == 1000 - 1000 % 512  # ReadOpChecksumInfoProto.chunkOffset
    first = packets[0][0]
    assert first["offset"] == 512 and first["offset"] <= 1000
    end = packets[-2][0]["offset"] + packets[-2][0]["data_len"]
    assert end >= 6000 and end % 512 == 0


def test_unknown_block_is_an_error_response(datanode):
    lb, port, add = datanode
    c = Conn(port)
    resp, packets = c.read_block(999_999, 0, 10)
    c.close()
    assert resp[1][0] != 0 and not packets


def test_status_reaches_datanode(datanode):
    lb, port, add = datanode
    data = splitmix_bytes(70_000, 3)
    add(55, data, 512)
    c = Conn(port)
    c.read_block(55, 0, data.nbytes)
    c.send_status(6)
    c.close()
    assert lb.last_status(wait_for=6) == 6  # DT_PROTO_CHECKSUM_OK


@pytest.mark.parametrize("engine", ["reference", "hw", "pcl"])
@pytest.mark.parametrize("bpc", [512, 4096, 513])
def test_reference_read_loop_baseline(datanode, engine, bpc):
    """bench.py's config-5 CPU baseline (tests/loopback.reference_read_block over oracle/remote_loop.h):
    RemoteBlockReader's receive -> verifyChecksum -> copy loop on one thread, with the reference's own
    HWCrc32c (oracle/_ref) or the restated engines. Clean blocks arrive byte for byte with CHECKSUM_OK
    sent; a flipped bit stops it at its packet (ChecksumException); verify off delivers the bytes as
    they came; a short tail's mismatch is ignored (RemoteBlockReader.cpp:319)."""
    from loopback import reference_read_block
    from util import ref_lib

    if engine == "reference" and ref_lib() is None:
        pytest.skip("oracle/_ref was not built (no /root/reference here)")
    dn, port, add = datanode
    n = (3 << 20) + 777
    data = splitmix_bytes(n, 900 + bpc)
    bid = 80_000 + bpc * 10 + ["reference", "hw", "pcl"].index(engine)
    crc = add(bid, data, bpc)
    out = np.zeros(n, np.uint8)
    assert reference_read_block(port, bid, n, out, engine=engine) == n
    assert np.array_equal(out, data)
    assert dn.last_status(wait_for=6) == 6
    per = max(bpc, 65536 // bpc * bpc)
    bad = data.copy()
    bad[20 * per + 5] ^= 0x08
    add(bid + 100_000, bad, bpc, crc=crc)
    with pytest.raises(OSError, match=r"ChecksumException: block \d+ packet 20"):
        reference_read_block(port, bid + 100_000, n, out, engine=engine)
    out[:] = 0
    assert reference_read_block(port, bid + 100_000, n, out, verify=False, engine=engine) == n
    assert np.array_equal(out, bad)
    tail = crc.copy()
    tail[-4] ^= 0xFF
    add(bid + 200_000, data, bpc, crc=tail)
    assert reference_read_block(port, bid + 200_000, n, out, engine=engine) == n
