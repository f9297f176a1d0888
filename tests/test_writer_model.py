"""CPU tests pinning the write-path packet model (tests/writer_model.py) to the reference's
stated numbers and to the oracle: chunks per packet 127/32/16 at
512/2048/4096 B chunks, a 65 563-byte full packet at 512, BE CRC words, the 31-byte header,
flush re-sending the partial chunk, and the empty last packet at every block boundary."""
import struct

import numpy as np
import pytest

from dtp import parse_packet_header
from util import oracle_crc, splitmix_bytes
from writer_model import OutputStreamModel


def crc(b: bytes) -> int:
    return oracle_crc(np.frombuffer(b, np.uint8)) if b else 0


@pytest.mark.parametrize("bpc,per", [(512, 127), (2048, 32), (4096, 16)])
def test_chunks_per_packet(bpc, per):
    m = OutputStreamModel(crc, bpc=bpc)
    assert m.chunks_per_packet == per
    data = splitmix_bytes(per * bpc, 1).tobytes()
    m.write(data)
    assert len(m.sent) == 1
    pkt, info = m.sent[0]
    assert info["num_chunks"] == per and info["data_len"] == per * bpc
    if bpc == 512:
        assert len(pkt) == 65563
    h = parse_packet_header(pkt[:31])
    assert h == {"packet_len": per * (bpc + 4) + 4, "offset": 0, "seqno": 0, "last": False, "data_len": per * bpc}
    words = struct.unpack(f">{per}I", pkt[31:31 + 4 * per])
    assert list(words) == [crc(data[i * bpc:(i + 1) * bpc]) for i in range(per)]


def test_flush_resends_partial_chunk_and_close_ends_block():
    m = OutputStreamModel(crc, bpc=512)
    data = splitmix_bytes(2000, 2).tobytes()
    m.write(data[:700])
    m.flush()
    m.write(data[700:])
    m.close()
    hdrs = [parse_packet_header(p[:31]) for p, _ in m.sent]
    # packet 0: chunk 0 + partial chunk 1 (188 B); packet 1 restarts at chunk 1
    assert [h["offset"] for h in hdrs] == [0, 512, 1536]
    assert [h["data_len"] for h in hdrs] == [700, 1488, 0]
    assert [h["seqno"] for h in hdrs] == [0, 1, 2] and hdrs[-1]["last"]


def test_empty_file_sends_nothing():
    m = OutputStreamModel(crc)
    m.close()
    assert m.sent == []


# ---- append (OutputStreamImpl::initAppend, OutputStreamImpl.cpp:172-230, 332-337) ----------------

def test_append_mid_chunk_first_packet_is_one_partial_chunk():
    """A file ending mid-chunk: the first packet holds exactly chunkSize - len % chunkSize bytes as
    ONE chunk whose CRC covers those bytes only, at offsetInBlock = the last block's length; the
    configured sizes return after it (127 chunks per packet again)."""
    bs = 1 << 20
    flen = 3 * bs + 5 * 512 + 100  # 100 bytes into a chunk of the 4th block
    m = OutputStreamModel(crc, bpc=512, block_size=bs, append=(flen, 5 * 512 + 100))
    assert (m.chunk_size, m.chunks_per_packet, m.packet_size) == (412, 1, 31 + 416)
    data = splitmix_bytes(412 + 127 * 512 + 10, 9).tobytes()
    m.write(data)
    m.close()
    (p0, i0), (p1, i1) = m.sent[0], m.sent[1]
    assert i0 == {"seqno": 0, "offset_in_block": 5 * 512 + 100, "block_index": 0, "data_len": 412,
                  "num_chunks": 1, "last": False}
    assert struct.unpack(">I", p0[31:35])[0] == crc(data[:412]) and p0[35:] == data[:412]
    assert i1["offset_in_block"] == 6 * 512 and i1["num_chunks"] == 127 and i1["data_len"] == 127 * 512
    # the empty last packet sits at bytesWritten, which counts whole chunks only
    assert m.sent[-1][1]["last"] and m.sent[-1][1]["offset_in_block"] == 6 * 512 + 127 * 512
    assert m.cursor == flen + len(data)


def test_append_mid_chunk_flush_before_the_chunk_fills():
    """hflush inside the partial chunk: a one-chunk packet of what was written, sent again (with
    the rest) once the chunk fills; the append sizes hold until that full packet."""
    m = OutputStreamModel(crc, bpc=512, block_size=1 << 20, append=(1048, 1048))  # 24 used, 488 free
    data = splitmix_bytes(600, 4).tobytes()
    m.write(data[:50])
    m.flush()
    m.write(data[50:])
    m.close()
    infos = [i for _, i in m.sent]
    assert [(i["offset_in_block"], i["data_len"], i["num_chunks"], i["last"]) for i in infos] == [
        (1048, 50, 1, False), (1048, 488, 1, False), (1536, 112, 1, False), (1536, 0, 0, True)]
    assert m.sent[1][0][35:] == data[:488]
    assert struct.unpack(">I", m.sent[1][0][31:35])[0] == crc(data[:488])


def test_append_on_chunk_boundary_caps_the_first_packet_at_the_free_space():
    """A file ending on a chunk boundary: packetSize = min(packetSize, freeInLastBlock)."""
    bs = 1 << 20
    m = OutputStreamModel(crc, bpc=512, block_size=bs, append=(2 * bs - 1024, bs - 1024))
    assert (m.chunk_size, m.chunks_per_packet) == (512, 2)  # (1024 - 31 + 515) // 516
    data = splitmix_bytes(5000, 6).tobytes()
    m.write(data)
    m.close()
    infos = [i for _, i in m.sent]
    # 2 chunks fill the block: its packet, its empty last packet, then a new block from offset 0
    assert [(i["block_index"], i["offset_in_block"], i["data_len"], i["last"]) for i in infos] == [
        (0, bs - 1024, 1024, False), (0, bs, 0, True), (1, 0, 5000 - 1024, False), (1, 7 * 512, 0, True)]


def test_append_without_last_block_starts_a_new_block():
    m = OutputStreamModel(crc, bpc=512, block_size=1 << 20, append=(2 << 20, -1))
    m.write(b"x" * 10)
    m.close()
    assert [(i["block_index"], i["offset_in_block"], i["data_len"]) for _, i in m.sent] == [(0, 0, 10), (0, 0, 0)]
    assert m.cursor == (2 << 20) + 10


def test_append_to_a_full_last_block_is_refused():
    with pytest.raises(IOError):
        OutputStreamModel(crc, bpc=512, block_size=1 << 20, append=(1 << 20, 1 << 20))
