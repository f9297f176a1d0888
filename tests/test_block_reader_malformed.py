"""GPU tests: the block reader against a scripted, misbehaving datanode (tests/dtp.serve_once).
Every malformed exchange must end in a clean error — never a crash, hang, huge allocation
or delivered garbage. Cases follow the checks of RemoteBlockReader::checkResponse
(:112-203), readNextPacket (:226-277) and PacketHeader::sanityCheck (PacketHeader.cpp:72-86),
plus two bounds the reference leaves to asserts (packet size, offset continuity)."""
import struct

import numpy as np
import pytest

from dtp import block_op_response, packet_header, serve_once, varint
from util import oracle_compute, splitmix_bytes

pytestmark = pytest.mark.gpu

DATA = splitmix_bytes(4096, 99)
CRC = oracle_compute(DATA, 512).tobytes()


def pkt(data: bytes, crc: bytes, offset: int, seqno: int, last=False, packet_len=None, data_len=None):
    dl = len(data) if data_len is None else data_len
    pl = 4 + len(data) + len(crc) if packet_len is None else packet_len
    return packet_header(pl, offset, seqno, last, dl) + crc + data


GOOD = pkt(DATA.tobytes(), CRC, 0, 0)
TRAILER = packet_header(4, 4096, 1, True, 0)


def attempt(script, start=0, length=4096, received=None):
    from libhdfs3_amd.engine import BlockReader
    from libhdfs3_amd._native import Hdfs3CrcError

    port, t = serve_once(script, received)
    try:
        with BlockReader("127.0.0.1", port, 1, start, length, timeout_ms=3000) as r:
            out = r.read_all(length)
        return out, None
    except Hdfs3CrcError as e:
        return None, e
    finally:
        t.join(10)


def test_well_formed_script_reads():
    out, err = attempt(lambda req: block_op_response() + GOOD + TRAILER)
    assert err is None and out.tobytes() == DATA.tobytes()


@pytest.mark.parametrize("name,script", [
    ("error status", lambda req: block_op_response(status=1)),
    ("unknown checksum type", lambda req: block_op_response(ctype=7)),
    ("chunk offset after start", lambda req: block_op_response(chunk_offset=512)),
    ("zero chunk size", lambda req: block_op_response(bpc=0)),
    ("garbage response", lambda req: varint(5) + b"\xff\xff\xff\xff\xff"),
    ("closed before response", lambda req: b""),
])
def test_bad_response_fails_open(name, script):
    out, err = attempt(script)
    assert err is not None, name


@pytest.mark.parametrize("name,script", [
    ("packetLen mismatch", lambda req: block_op_response() + pkt(DATA.tobytes(), CRC, 0, 0, packet_len=999)),
    ("seqno does not start at 0", lambda req: block_op_response() + pkt(DATA.tobytes(), CRC, 0, 1)),
    ("empty non-last packet", lambda req: block_op_response() + packet_header(4, 0, 0, False, 0)),
    ("last packet with data", lambda req: block_op_response() + pkt(DATA.tobytes(), CRC, 0, 0, last=True)),
    ("1 GiB dataLen", lambda req: block_op_response() + packet_header(4 + (1 << 30) + 4 * (1 << 21), 0, 0, False,
                                                                     1 << 30)),
    ("offset gap", lambda req: block_op_response() + pkt(DATA.tobytes(), CRC, 4096, 0)),
    ("truncated payload", lambda req: block_op_response() + GOOD[:1000]),
    ("negative dataLen", lambda req: block_op_response() + packet_header(4, 0, 0, False, -5)),
])
def test_bad_packets_fail_cleanly(name, script):
    out, err = attempt(script)
    assert err is not None and out is None, name


def test_corrupt_crc_is_checksum_exception():
    bad = bytearray(CRC)
    bad[5] ^= 1  # chunk 1
    out, err = attempt(lambda req: block_op_response() + pkt(DATA.tobytes(), bytes(bad), 0, 0) + TRAILER)
    assert err is not None and "ChecksumException" in str(err)


def test_status_only_after_the_empty_trailer():
    """sendStatus runs only when readTrailingEmptyPacket sees {lastPacketInBlock, dataLen 0}
    (RemoteBlockReader.cpp:274-286): CHECKSUM_OK (status 6) after a proper trailer; nothing
    when the datanode keeps streaming a data packet after the range."""
    got = []
    out, err = attempt(lambda req: block_op_response() + GOOD + TRAILER, received=got)
    assert err is None and out.tobytes() == DATA.tobytes()
    msg = b"".join(got)
    assert msg == varint(2) + bytes([0x08, 6]), msg  # ClientReadStatusProto{status: CHECKSUM_OK}
    got = []
    more = pkt(DATA.tobytes(), CRC, 4096, 1)  # a data packet where the trailer belongs
    out, err = attempt(lambda req: block_op_response() + GOOD + more, received=got)
    assert err is None and out.tobytes() == DATA.tobytes()
    assert b"".join(got) == b""


@pytest.mark.parametrize("bpc", [1, 3, 513, 517])
def test_any_positive_chunk_size(bpc):
    """RemoteBlockReader accepts any bytesPerChecksum > 0 from the datanode (:150-156); the
    remote rule still ignores a short-tail mismatch (:319)."""
    n = 4096
    crc = oracle_compute(DATA[:n], bpc).tobytes()
    script = lambda req: block_op_response(bpc=bpc) + pkt(DATA.tobytes(), crc, 0, 0) + TRAILER
    out, err = attempt(script)
    assert err is None and out.tobytes() == DATA.tobytes(), err
    bad = bytearray(crc)
    k = 1000 // bpc if bpc > 4 else 7
    bad[4 * k] ^= 1
    out, err = attempt(lambda req: block_op_response(bpc=bpc) + pkt(DATA.tobytes(), bytes(bad), 0, 0) + TRAILER)
    assert err is not None and "ChecksumException" in str(err)
    if n % bpc:  # a bad word on the short tail chunk is ignored remotely
        tail = bytearray(crc)
        tail[-1] ^= 1
        out, err = attempt(lambda req: block_op_response(bpc=bpc) + pkt(DATA.tobytes(), bytes(tail), 0, 0) + TRAILER)
        assert err is None and out.tobytes() == DATA.tobytes()
