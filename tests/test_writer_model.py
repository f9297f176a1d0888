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
