"""Independent Python restatement of the HDFS data-transfer wire formats used on the
checksum path (test infrastructure): the client side of RemoteBlockReader
(src/client/RemoteBlockReader.cpp:46-357), DataTransferProtocolSender framing
(DataTransferProtocolSender.cpp:42-57,107-123) and PacketHeader
(src/client/PacketHeader.cpp:38-123). Used to cross-check the C++ codec and the
loopback datanode without a GPU."""
from __future__ import annotations

import socket
import struct


def varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def field_varint(f: int, v: int) -> bytes:
    return varint(f << 3) + varint(v)


def field_bytes(f: int, b: bytes) -> bytes:
    return varint((f << 3) | 2) + varint(len(b)) + b


def parse(buf: bytes) -> dict:
    """Minimal protobuf parser -> {field: [values]} (bytes for wiretype 2)."""
    out, i = {}, 0
    while i < len(buf):
        key, i = _rd_varint(buf, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _rd_varint(buf, i)
        elif wt == 1:
            v = struct.unpack_from("<q", buf, i)[0]
            i += 8
        elif wt == 5:
            v = struct.unpack_from("<i", buf, i)[0]
            i += 4
        elif wt == 2:
            n, i = _rd_varint(buf, i)
            v = buf[i:i + n]
            i += n
        else:
            raise ValueError(f"wiretype {wt}")
        out.setdefault(f, []).append(v)
    return out


def _rd_varint(buf: bytes, i: int):
    v = shift = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return v, i


def read_block_request(block_id: int, offset: int, length: int, pool: bytes = b"BP-test",
                       client: bytes = b"pytest") -> bytes:
    eb = field_bytes(1, pool) + field_varint(2, block_id) + field_varint(3, 1) + field_varint(4, 0)
    token = field_bytes(1, b"") + field_bytes(2, b"") + field_bytes(3, b"") + field_bytes(4, b"")
    base = field_bytes(1, eb) + field_bytes(2, token)
    header = field_bytes(1, base) + field_bytes(2, client)
    op = field_bytes(1, header) + field_varint(2, offset) + field_varint(3, length)
    return struct.pack(">hB", 28, 81) + varint(len(op)) + op


def packet_header(packet_len: int, offset: int, seqno: int, last: bool, data_len: int) -> bytes:
    """31-byte header as Packet::getBuffer writes it (Packet.cpp:124-153)."""
    proto = (b"\x09" + struct.pack("<q", offset) + b"\x11" + struct.pack("<q", seqno) +
             b"\x18" + bytes([1 if last else 0]) + b"\x25" + struct.pack("<i", data_len))
    assert len(proto) == 25
    return struct.pack(">ih", packet_len, len(proto)) + proto


def parse_packet_header(b: bytes):
    packet_len, proto_len = struct.unpack_from(">ih", b, 0)
    f = parse(b[6:6 + proto_len])
    return {"packet_len": packet_len, "offset": f[1][0], "seqno": f[2][0], "last": bool(f[3][0]),
            "data_len": f[4][0]}


class Conn:
    def __init__(self, port: int):
        self.s = socket.create_connection(("127.0.0.1", port), timeout=30)

    def recv_exact(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.s.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("peer closed")
            buf += chunk
        return bytes(buf)

    def recv_delimited(self) -> bytes:
        v = shift = 0
        while True:
            b = self.recv_exact(1)[0]
            v |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
        return self.recv_exact(v)

    def read_block(self, block_id: int, offset: int, length: int):
        """Full RemoteBlockReader exchange; returns (response fields, [(header, crc_bytes, data)])."""
        self.s.sendall(read_block_request(block_id, offset, length))
        resp = parse(self.recv_delimited())
        if resp[1][0] != 0:
            return resp, []
        info = parse(resp[4][0])
        cs = parse(info[1][0])
        bpc = cs[2][0]
        packets = []
        while True:
            h = parse_packet_header(self.recv_exact(31))
            if h["data_len"] == 0:
                assert h["last"]
                packets.append((h, b"", b""))
                break
            chunks = (h["data_len"] + bpc - 1) // bpc
            payload = self.recv_exact(4 * chunks + h["data_len"])
            packets.append((h, payload[:4 * chunks], payload[4 * chunks:]))
        return resp, packets

    def send_status(self, status: int) -> None:
        msg = field_varint(1, status)
        self.s.sendall(varint(len(msg)) + msg)

    def close(self):
        self.s.close()


def serve_once(script, received=None):
    """Test helper: a one-connection fake datanode on 127.0.0.1. After reading the client's
    OP_READ_BLOCK request it sends the bytes `script(request_fields)` returns, then keeps
    the socket open until the client goes away, appending whatever the client sends after
    the request (its ClientReadStatusProto) to the list `received`. Returns (port, thread)."""
    import threading

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def run():
        c, _ = srv.accept()
        try:
            c.settimeout(10)
            hdr = b""
            while len(hdr) < 3:
                hdr += c.recv(3 - len(hdr))
            n = shift = 0
            while True:
                b = c.recv(1)[0]
                n |= (b & 0x7F) << shift
                shift += 7
                if not b & 0x80:
                    break
            body = b""
            while len(body) < n:
                body += c.recv(n - len(body))
            c.sendall(script(parse(body)))
            try:
                while True:
                    got = c.recv(65536)
                    if not got:
                        break
                    if received is not None:
                        received.append(got)
            except OSError:
                pass
        finally:
            c.close()
            srv.close()

    t = threading.Thread(target=run, daemon=True)
    t.start()
    return port, t


def block_op_response(bpc: int = 512, ctype: int = 2, chunk_offset: int = 0, status: int = 0) -> bytes:
    """BlockOpResponseProto{status, readOpChecksumInfo{checksum{type, bpc}, chunkOffset}}, delimited."""
    cs = field_varint(1, ctype) + field_varint(2, bpc)
    info = field_bytes(1, cs) + field_varint(2, chunk_offset)
    msg = field_varint(1, status) + field_bytes(4, info)
    return varint(len(msg)) + msg
