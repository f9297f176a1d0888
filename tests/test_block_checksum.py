"""Block checksum, "MD5 of CRC32" (OP_BLOCK_CHECKSUM).

The reference declares the op (DataTransferProtocolSender.h:49, :112-120) and leaves its
body a TODO (DataTransferProtocolSender.cpp:169-180); the reply it would parse is
OpBlockChecksumResponseProto {bytesPerCrc, crcPerBlock, md5, crcType}
(datatransfer.proto:222-227), md5 being the digest of the block's stored big-endian CRC
words. No reference test covers it, so parity is pinned by pieces that are: the CRC words
by the oracle (itself pinned by the reference KATs), MD5 by hashlib (RFC 1321), and the
framing by the independent Python codec in tests/dtp.py.

CPU tests: MD5 over held CRC words, the file checksum, the loopback datanode's answer
through an independent client, and the product client against the loopback datanode and
against scripted fake datanodes. GPU tests: hdfs3_block_checksum_dev (GPU CRC words, host
MD5) against hashlib over the oracle's words, and end to end against the datanode.
"""
import errno
import hashlib
import struct

import numpy as np
import pytest

from dtp import Conn, field_bytes, field_varint, parse, serve_once, varint
from util import oracle_compute, oracle_compute_crc32, splitmix_bytes


def md5_of_crcs(crc_be: np.ndarray) -> bytes:
    return hashlib.md5(np.ascontiguousarray(crc_be).tobytes()).digest()


@pytest.fixture(scope="module")
def datanode():
    from loopback import LoopbackDatanode

    dn = LoopbackDatanode()
    yield dn
    dn.stop()


# ---- CPU ---------------------------------------------------------------------------

@pytest.mark.parametrize("n_words", [0, 1, 13, 14, 15, 16, 17, 31, 32, 33, 1000, 262144])
def test_md5_of_held_crcs_matches_hashlib(n_words):
    # 13..17 and 31..33 words put the message end on both sides of MD5's 56/64-byte padding edges
    from libhdfs3_amd.engine import block_checksum_crcs

    words = splitmix_bytes(4 * n_words, 0xC0FFEE + n_words)
    assert block_checksum_crcs(words) == hashlib.md5(words.tobytes()).digest()


def test_md5_known_answers():
    # RFC 1321 appendix A.5 strings whose length is a multiple of 4 (the API takes CRC words)
    from libhdfs3_amd.engine import block_checksum_crcs

    assert block_checksum_crcs(b"").hex() == "d41d8cd98f00b204e9800998ecf8427e"
    digits = b"1234567890" * 8
    assert block_checksum_crcs(digits).hex() == "57edf4a22be3c955ac49da2e2107b67a"


def test_file_checksum_is_md5_of_block_digests():
    from libhdfs3_amd.engine import block_checksum_crcs, file_checksum_md5md5crc

    blocks = [block_checksum_crcs(splitmix_bytes(4 * n, n)) for n in (256, 2048, 7)]
    assert file_checksum_md5md5crc(blocks) == hashlib.md5(b"".join(blocks)).digest()
    assert file_checksum_md5md5crc([]) == hashlib.md5(b"").digest()


def _block_checksum_request(block_id: int, pool: bytes = b"BP-test") -> bytes:
    eb = field_bytes(1, pool) + field_varint(2, block_id) + field_varint(3, 1) + field_varint(4, 0)
    token = field_bytes(1, b"") + field_bytes(2, b"") + field_bytes(3, b"") + field_bytes(4, b"")
    op = field_bytes(1, field_bytes(1, eb) + field_bytes(2, token))
    return struct.pack(">hB", 28, 85) + varint(len(op)) + op


@pytest.mark.parametrize("bpc,nbytes,ctype", [(512, 1 << 20, 2), (4096, (1 << 20) + 300, 2),
                                               (512, 64 * 1024 - 100, 1)])
def test_loopback_datanode_answers_block_checksum(datanode, bpc, nbytes, ctype):
    """Independent client (tests/dtp.py framing) against the loopback datanode."""
    data = splitmix_bytes(nbytes, bpc + ctype)
    crc = oracle_compute(data, bpc) if ctype == 2 else oracle_compute_crc32(data, bpc)
    bid = 7000 + bpc + ctype
    datanode.add_block(bid, data, crc, bpc, ctype)
    c = Conn(datanode.port)
    try:
        c.s.sendall(_block_checksum_request(bid))
        resp = parse(c.recv_delimited())
    finally:
        c.close()
    assert resp[1] == [0]
    cr = parse(resp[3][0])
    assert cr[1] == [bpc] and cr[2] == [(nbytes + bpc - 1) // bpc] and cr[4] == [ctype]
    assert cr[3][0] == md5_of_crcs(crc)


@pytest.mark.parametrize("bpc,nbytes", [(512, 1 << 20), (2048, 3 * 2048 + 17)])
def test_remote_client_against_loopback(datanode, bpc, nbytes):
    from libhdfs3_amd.engine import block_checksum_remote

    data = splitmix_bytes(nbytes, 99 + bpc)
    crc = oracle_compute(data, bpc)
    bid = 8000 + bpc
    datanode.add_block(bid, data, crc, bpc)
    got_bpc, n, md5, ctype = block_checksum_remote("127.0.0.1", datanode.port, bid)
    assert (got_bpc, n, ctype) == (bpc, (nbytes + bpc - 1) // bpc, 2)
    assert md5 == md5_of_crcs(crc)


def test_remote_client_errors(datanode):
    from libhdfs3_amd._native import Hdfs3CrcError
    from libhdfs3_amd.engine import block_checksum_remote

    with pytest.raises(Hdfs3CrcError) as e:  # status ERROR_INVALID: block not found
        block_checksum_remote("127.0.0.1", datanode.port, 123456789)
    assert e.value.rc == -errno.EIO and "block not found" in str(e.value)
    data = splitmix_bytes(4096, 1)
    datanode.add_block(8999, data, None, 512, 0)  # CHECKSUM_NULL block has no CRC words
    with pytest.raises(Hdfs3CrcError) as e:
        block_checksum_remote("127.0.0.1", datanode.port, 8999)
    assert e.value.rc == -errno.EIO


def _checksum_response(md5: bytes, bpc=512, n=2, ctype=None, status=0) -> bytes:
    cr = field_varint(1, bpc) + field_varint(2, n) + field_bytes(3, md5)
    if ctype is not None:
        cr += field_varint(4, ctype)
    msg = field_varint(1, status) + field_bytes(3, cr)
    return varint(len(msg)) + msg


def test_remote_client_request_fields_and_reply_parsing():
    """Scripted datanode: the request carries the block in BaseHeaderProto; the reply's
    fields come back unchanged, with crcType optional."""
    from libhdfs3_amd.engine import block_checksum_remote

    seen = {}
    md5 = bytes(range(16))

    def script(req):
        base = parse(req[1][0])
        eb = parse(base[1][0])
        seen.update(pool=eb[1][0], block=eb[2][0], gs=eb[3][0], token=parse(base[2][0]))
        return _checksum_response(md5, bpc=4096, n=33)

    port, t = serve_once(script)
    assert block_checksum_remote("127.0.0.1", port, 42, pool_id=b"BP-x", generation_stamp=9) == \
        (4096, 33, md5, -1)
    t.join(5)
    assert seen["pool"] == b"BP-x" and seen["block"] == 42 and seen["gs"] == 9
    assert sorted(seen["token"]) == [1, 2, 3, 4]


@pytest.mark.parametrize("reply,err", [
    (lambda: _checksum_response(bytes(16), status=1), errno.EIO),          # ERROR
    (lambda: varint(2) + field_varint(1, 0), errno.EIO),                   # SUCCESS without checksumResponse
    (lambda: _checksum_response(bytes(15)), errno.EPROTO),                 # md5 of the wrong size
    (lambda: varint(3) + b"\x0a\xff\xff", errno.EPROTO),                   # unparseable proto
])
def test_remote_client_rejects_bad_replies(reply, err):
    from libhdfs3_amd._native import Hdfs3CrcError
    from libhdfs3_amd.engine import block_checksum_remote

    port, t = serve_once(lambda req: reply())
    with pytest.raises(Hdfs3CrcError) as e:
        block_checksum_remote("127.0.0.1", port, 1, timeout_ms=5000)
    assert e.value.rc == -err
    t.join(5)


# ---- GPU ---------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("bpc", [512, 2048, 4096])
@pytest.mark.parametrize("nbytes", [1, 300, 64 * 1024 * 16 + 300, 128 << 20])
def test_block_checksum_dev_matches_oracle(bpc, nbytes):
    from libhdfs3_amd.engine import CrcContext

    data = splitmix_bytes(nbytes, nbytes ^ bpc)
    with CrcContext(0) as ctx:
        d = ctx.upload(data)
        md5, n = ctx.block_checksum_dev(d.ptr, nbytes, bpc)
    assert n == (nbytes + bpc - 1) // bpc
    assert md5 == md5_of_crcs(oracle_compute(data, bpc))


@pytest.mark.gpu
def test_block_checksum_dev_pieces_and_empty():
    """More than one 1 Mi-chunk piece (bpc 4: 2.6 Mi chunks, three pieces through both
    slots), and the empty block (MD5 of nothing, crcPerBlock 0)."""
    from libhdfs3_amd.engine import CrcContext

    nbytes = (10 << 20) + 8
    data = splitmix_bytes(nbytes, 4)
    with CrcContext(0) as ctx:
        d = ctx.upload(data)
        md5, n = ctx.block_checksum_dev(d.ptr, nbytes, 4)
        assert (md5, n) == (md5_of_crcs(oracle_compute(data, 4)), nbytes // 4)
        assert ctx.block_checksum_dev(d.ptr, 0, 512) == (hashlib.md5(b"").digest(), 0)
        assert ctx.kernel_launches >= 3


@pytest.mark.gpu
def test_block_checksum_dev_crc32_type():
    from libhdfs3_amd.engine import CrcContext

    data = splitmix_bytes((1 << 20) + 44, 32)
    with CrcContext(0) as ctx:
        ctx.set_checksum_type(1)
        d = ctx.upload(data)
        md5, _ = ctx.block_checksum_dev(d.ptr, data.nbytes, 512)
    assert md5 == md5_of_crcs(oracle_compute_crc32(data, 512))


@pytest.mark.gpu
def test_replica_block_checksums_match_datanode_end_to_end(datanode):
    """A writer's GPU CRC words served by the datanode; its OP_BLOCK_CHECKSUM answer equals
    the GPU block checksum of the same bytes, and the file checksum follows."""
    from libhdfs3_amd.engine import CrcContext, block_checksum_remote, file_checksum_md5md5crc

    sizes = [8 << 20, 8 << 20, (3 << 20) + 1000]
    digests = []
    with CrcContext(0) as ctx:
        for i, nbytes in enumerate(sizes):
            data = splitmix_bytes(nbytes, 500 + i)
            crc = ctx.compute(data, 512)
            datanode.add_block(9100 + i, data, crc, 512)
            d = ctx.upload(data)
            md5, n = ctx.block_checksum_dev(d.ptr, nbytes, 512)
            remote = block_checksum_remote("127.0.0.1", datanode.port, 9100 + i)
            assert remote == (512, n, md5, 2)
            digests.append(md5)
    assert file_checksum_md5md5crc(digests) == hashlib.md5(
        b"".join(md5_of_crcs(oracle_compute(splitmix_bytes(s, 500 + i), 512)) for i, s in enumerate(sizes))
    ).digest()
