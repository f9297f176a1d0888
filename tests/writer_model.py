"""Test infrastructure: a pure-Python restatement of the reference's write-path packet
production — OutputStreamImpl::computePacketChunkSize / initAppend / appendInternal /
appendChunkToPacket / flushInternal / closePipeline / close (src/client/OutputStreamImpl.cpp:
161-230, 298-359, 392-431, 512-575)
and Packet::addChecksum / addData / getBuffer (src/client/Packet.cpp:44-153) — with the
pipeline replaced by a list of sent packets. CRCs come from the oracle (crc32c), so this
is the packet-level oracle the GPU output stream is checked against byte for byte."""
from __future__ import annotations

import struct

HEADER = 31


def packet_header(packet_len: int, offset: int, seqno: int, last: bool, data_len: int) -> bytes:
    """PacketHeader::writeInBuffer (PacketHeader.cpp:100-123)."""
    proto = (b"\x09" + struct.pack("<q", offset) + b"\x11" + struct.pack("<q", seqno) +
             b"\x18" + bytes([1 if last else 0]) + b"\x25" + struct.pack("<i", data_len))
    return struct.pack(">ih", packet_len, len(proto)) + proto


class _Packet:
    def __init__(self, offset: int, seqno: int, max_chunks: int):
        self.offset, self.seqno, self.max_chunks = offset, seqno, max_chunks
        self.sums: list[int] = []
        self.data = bytearray()
        self.last = False

    def add(self, crc: int, data: bytes) -> None:  # addChecksum + addData + increaseNumChunks
        self.sums.append(crc)
        self.data += data

    def full(self) -> bool:
        return len(self.sums) >= self.max_chunks

    def buffer(self) -> bytes:  # getBuffer
        sums = b"".join(struct.pack(">I", c) for c in self.sums)
        return packet_header(len(self.data) + len(sums) + 4, self.offset, self.seqno, self.last,
                             len(self.data)) + sums + bytes(self.data)


def chunks_per_packet(packet_size: int, chunk_size: int) -> tuple[int, int]:
    """computePacketChunkSize (OutputStreamImpl.cpp:161-170): (chunksPerPacket, packetSize).
    C++ integer division truncates toward zero (packetSize may be 0 in initAppend)."""
    with_sum = chunk_size + 4
    num = packet_size - HEADER + with_sum - 1
    n = max(1, int(num / with_sum) if num < 0 else num // with_sum)
    return n, n * with_sum + HEADER


class OutputStreamModel:
    def __init__(self, crc32c, bpc: int = 512, packet_size: int = 65536, block_size: int = 64 << 20,
                 append: tuple[int, int] | None = None):
        """append = (file_length, last_block_bytes) runs initAppend (OutputStreamImpl.cpp:172-230)
        for a file whose last block holds last_block_bytes (-1: the namenode returned no last
        block, i.e. the file ends on a block boundary)."""
        self.crc32c = crc32c  # bytes -> int (the oracle)
        self.bpc = bpc
        self.default_packet_size = packet_size
        self.chunk_size = bpc
        self.chunks_per_packet, self.packet_size = chunks_per_packet(packet_size, bpc)
        self.block_size = block_size
        self.buffer = bytearray()  # the chunk buffer (`buffer`, `position`)
        self.cursor = self.last_flushed = self.bytes_written = self.next_seqno = 0
        self.block_index = 0
        self.current: _Packet | None = None
        self.pipeline = False
        self.is_append = False
        self.sent: list[tuple[bytes, dict]] = []
        if append is not None:
            self._init_append(*append)

    def _init_append(self, file_length: int, last_block_bytes: int) -> None:
        self.cursor = self.last_flushed = file_length
        if last_block_bytes < 0:  # no last block: the next write starts a new block
            return
        self.is_append = True
        self.bytes_written = last_block_bytes
        free_in_block = self.block_size - file_length % self.block_size
        if free_in_block == self.block_size:
            raise IOError("OutputStreamImpl: the last block is full.")
        used_in_cksum = file_length % self.chunk_size
        free_in_cksum = self.chunk_size - used_in_cksum
        packet_size = self.default_packet_size
        if used_in_cksum > 0 and free_in_cksum > 0:
            # the next packet has exactly one chunk, filling up the partial chunk
            packet_size = 0
            self.chunk_size = free_in_cksum
        else:
            packet_size = min(packet_size, free_in_block)
        self.chunks_per_packet, self.packet_size = chunks_per_packet(packet_size, self.chunk_size)

    def _append_chunk(self, data: bytes) -> None:  # appendChunkToPacket
        if self.current is None:
            self.current = _Packet(self.bytes_written, self.next_seqno, self.chunks_per_packet)
            self.next_seqno += 1
        self.current.add(self.crc32c(data), data)

    def _send(self) -> None:  # sendPacket -> PipelineImpl::send
        p = self.current
        self.pipeline = True
        self.sent.append((p.buffer(), {"seqno": p.seqno, "offset_in_block": p.offset,
                                       "block_index": self.block_index, "data_len": len(p.data),
                                       "num_chunks": len(p.sums), "last": p.last}))
        self.current = None

    def _close_pipeline(self) -> None:
        if not self.pipeline:
            return
        if self.current is not None:
            self._send()
        self.current = _Packet(self.bytes_written, self.next_seqno, self.chunks_per_packet)
        self.next_seqno += 1
        self.current.last = True
        self._send()
        self.pipeline = False
        self.bytes_written = 0
        self.block_index += 1

    def write(self, buf: bytes) -> None:  # appendInternal
        size, todo = len(buf), len(buf)
        while todo > 0:
            cs = self.chunk_size  # buffer.size()
            n = min(cs - len(self.buffer), todo)
            piece = buf[size - todo:size - todo + n]
            if not self.buffer and todo >= cs:  # bypass buffer
                self._append_chunk(piece)
                self.bytes_written += n
            else:
                self.buffer += piece
                if len(self.buffer) == cs:
                    self._append_chunk(bytes(self.buffer))
                    self.bytes_written += cs
                    self.buffer.clear()
            todo -= n
            if self.current is not None and (self.current.full() or self.bytes_written == self.block_size):
                self._send()
                if self.is_append:  # back to the configured chunk and packet sizes (:332-337)
                    self.is_append = False
                    self.chunk_size = self.bpc
                    self.chunks_per_packet, self.packet_size = chunks_per_packet(self.default_packet_size, self.bpc)
                if self.bytes_written == self.block_size:
                    self._close_pipeline()
        self.cursor += size

    def _flush(self, need_sync: bool) -> None:  # flushInternal
        if self.last_flushed == self.cursor and not need_sync:
            return
        self.last_flushed = self.cursor
        if self.buffer:
            self._append_chunk(bytes(self.buffer))
        if self.current is None and need_sync and self.pipeline:
            self.current = _Packet(self.bytes_written, self.next_seqno, self.chunks_per_packet)
            self.next_seqno += 1
        if self.current is not None:
            self._send()

    def flush(self) -> None:
        self._flush(False)

    def sync(self) -> None:
        self._flush(True)

    def close(self) -> None:
        if self.last_flushed != self.cursor and self.buffer:
            self._append_chunk(bytes(self.buffer))
        if self.last_flushed != self.cursor and self.current is not None:
            self._send()
        self._close_pipeline()
