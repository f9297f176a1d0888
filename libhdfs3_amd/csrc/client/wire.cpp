// Hand-encoded protobuf subset for the checksum path; see wire.h for the reference map.
#include "wire.h"

#include <cstring>

namespace hdfs3crc {
namespace wire {

void put_varint(std::string &out, uint64_t v) {
    while (v >= 0x80) {
        out.push_back(char(uint8_t(v) | 0x80));
        v >>= 7;
    }
    out.push_back(char(v));
}

void put_tag(std::string &out, int field, int wiretype) { put_varint(out, (uint64_t(field) << 3) | wiretype); }

void put_fixed64(std::string &out, uint64_t v) {
    for (int i = 0; i < 8; ++i) out.push_back(char(uint8_t(v >> (8 * i))));
}

void put_fixed32(std::string &out, uint32_t v) {
    for (int i = 0; i < 4; ++i) out.push_back(char(uint8_t(v >> (8 * i))));
}

void put_bytes(std::string &out, int field, const std::string &s) {
    put_tag(out, field, 2);
    put_varint(out, s.size());
    out += s;
}

void put_uint(std::string &out, int field, uint64_t v) {
    put_tag(out, field, 0);
    put_varint(out, v);
}

uint64_t Reader::varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
        if (p >= end) {
            ok = false;
            return 0;
        }
        const uint8_t b = *p++;
        v |= uint64_t(b & 0x7F) << shift;
        if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
}

uint64_t Reader::fixed64() {
    if (end - p < 8) {
        ok = false;
        return 0;
    }
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= uint64_t(p[i]) << (8 * i);
    p += 8;
    return v;
}

uint32_t Reader::fixed32() {
    if (end - p < 4) {
        ok = false;
        return 0;
    }
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) v |= uint32_t(p[i]) << (8 * i);
    p += 4;
    return v;
}

std::string Reader::bytes() {
    const uint64_t n = varint();
    if (!ok || uint64_t(end - p) < n) {
        ok = false;
        return {};
    }
    std::string s(reinterpret_cast<const char *>(p), size_t(n));
    p += n;
    return s;
}

void Reader::skip(int wiretype) {
    switch (wiretype) {
    case 0: varint(); break;
    case 1: fixed64(); break;
    case 2: bytes(); break;
    case 5: fixed32(); break;
    default: ok = false;
    }
}

// ---- PacketHeader -------------------------------------------------------------

void PacketHeader::encode(uint8_t out[kPacketHeaderSize]) const {
    std::string proto;
    put_tag(proto, 1, 1);
    put_fixed64(proto, uint64_t(offset_in_block));
    put_tag(proto, 2, 1);
    put_fixed64(proto, uint64_t(seqno));
    put_tag(proto, 3, 0);
    put_varint(proto, last_packet_in_block ? 1 : 0);
    put_tag(proto, 4, 5);
    put_fixed32(proto, uint32_t(data_len));
    wr_be32(out, uint32_t(packet_len));
    wr_be16(out + 4, uint16_t(proto.size()));
    std::memcpy(out + 6, proto.data(), proto.size());  // 25 bytes: total 31
}

bool PacketHeader::decode(const uint8_t *buf, size_t n) {
    if (n < 6) return false;
    packet_len = int32_t(rd_be32(buf));
    const int proto_len = int16_t(rd_be16(buf + 4));
    // PacketHeader.cpp:105-110: packetLen >= 4, protoLen >= 0, proto inside the buffer
    if (packet_len < 4 || proto_len < 0 || 6 + size_t(proto_len) > n) return false;
    Reader r(buf + 6, size_t(proto_len));
    bool seen[5] = {false, false, false, false, false};
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 1) offset_in_block = int64_t(r.fixed64()), seen[1] = true;
        else if (field == 2 && wt == 1) seqno = int64_t(r.fixed64()), seen[2] = true;
        else if (field == 3 && wt == 0) last_packet_in_block = r.varint() != 0, seen[3] = true;
        else if (field == 4 && wt == 5) data_len = int32_t(r.fixed32()), seen[4] = true;
        else if (field == 5 && wt == 0) sync_block = r.varint() != 0;
        else r.skip(wt);
    }
    // required fields (datatransfer.proto:144-148)
    return r.ok && seen[1] && seen[2] && seen[3] && seen[4];
}

bool PacketHeader::sanity_check(int64_t last_seqno) const {
    if (data_len <= 0 && !last_packet_in_block) return false;   // only the last may be empty
    if (last_packet_in_block && data_len != 0) return false;    // the last carries no data
    if (seqno != last_seqno + 1) return false;                  // seqnos increase by one
    return true;
}

// ---- requests / responses -----------------------------------------------------

static std::string encode_extended_block(const ExtendedBlock &b) {
    std::string s;
    put_bytes(s, 1, b.pool_id);
    put_uint(s, 2, b.block_id);
    put_uint(s, 3, b.generation_stamp);
    put_uint(s, 4, b.num_bytes);
    return s;
}

// BaseHeaderProto {1: block, 2: TokenProto} (datatransfer.proto:40-43); the token's four
// required fields are empty (security is out of scope)
static std::string encode_base_header(const ExtendedBlock &b) {
    std::string token;
    put_bytes(token, 1, "");
    put_bytes(token, 2, "");
    put_bytes(token, 3, "");
    put_bytes(token, 4, "");
    std::string base;
    put_bytes(base, 1, encode_extended_block(b));
    put_bytes(base, 2, token);
    return base;
}

static std::string frame_op(int op, const std::string &proto) {
    std::string out;
    out.push_back(char(kDataTransferVersion >> 8));
    out.push_back(char(kDataTransferVersion & 0xFF));
    out.push_back(char(op));
    put_varint(out, proto.size());
    out += proto;
    return out;
}

std::string encode_read_block(const ReadBlockRequest &r) {
    const std::string base = encode_base_header(r.block);
    std::string client_header;
    put_bytes(client_header, 1, base);
    put_bytes(client_header, 2, r.client_name);
    std::string op;
    put_bytes(op, 1, client_header);
    put_uint(op, 2, r.offset);
    put_uint(op, 3, r.len);
    if (!r.send_checksums) put_uint(op, 4, 0);
    return frame_op(kOpReadBlock, op);
}

std::string encode_block_checksum(const ExtendedBlock &block) {
    std::string op;
    put_bytes(op, 1, encode_base_header(block));
    return frame_op(kOpBlockChecksum, op);
}

static bool decode_extended_block(const std::string &s, ExtendedBlock &b) {
    Reader r(s.data(), s.size());
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 2) b.pool_id = r.bytes();
        else if (field == 2 && wt == 0) b.block_id = r.varint();
        else if (field == 3 && wt == 0) b.generation_stamp = r.varint();
        else if (field == 4 && wt == 0) b.num_bytes = r.varint();
        else r.skip(wt);
    }
    return r.ok;
}

bool decode_block_checksum(const void *proto, size_t n, ExtendedBlock &out) {
    Reader r(proto, n);
    bool have_block = false;
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 2) {
            const std::string base = r.bytes();
            Reader b(base.data(), base.size());
            while (b.more()) {
                const uint64_t k2 = b.varint();
                const int f2 = int(k2 >> 3), w2 = int(k2 & 7);
                if (f2 == 1 && w2 == 2) {
                    if (!decode_extended_block(b.bytes(), out)) return false;
                    have_block = true;
                } else {
                    b.skip(w2);
                }
            }
            if (!b.ok) return false;
        } else {
            r.skip(wt);
        }
    }
    return r.ok && have_block;
}

bool decode_read_block(const void *proto, size_t n, ReadBlockRequest &out) {
    Reader r(proto, n);
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 2) {
            const std::string ch = r.bytes();
            Reader h(ch.data(), ch.size());
            while (h.more()) {
                const uint64_t k2 = h.varint();
                const int f2 = int(k2 >> 3), w2 = int(k2 & 7);
                if (f2 == 1 && w2 == 2) {
                    const std::string base = h.bytes();
                    Reader b(base.data(), base.size());
                    while (b.more()) {
                        const uint64_t k3 = b.varint();
                        const int f3 = int(k3 >> 3), w3 = int(k3 & 7);
                        if (f3 == 1 && w3 == 2) {
                            if (!decode_extended_block(b.bytes(), out.block)) return false;
                        } else {
                            b.skip(w3);
                        }
                    }
                    if (!b.ok) return false;
                } else if (f2 == 2 && w2 == 2) {
                    out.client_name = h.bytes();
                } else {
                    h.skip(w2);
                }
            }
            if (!h.ok) return false;
        } else if (field == 2 && wt == 0) {
            out.offset = r.varint();
        } else if (field == 3 && wt == 0) {
            out.len = r.varint();
        } else if (field == 4 && wt == 0) {
            out.send_checksums = r.varint() != 0;
        } else {
            r.skip(wt);
        }
    }
    return r.ok;
}

std::string encode_block_op_response(const BlockOpResponse &r) {
    std::string out;
    put_uint(out, 1, uint64_t(r.status));
    if (!r.first_bad_link.empty()) put_bytes(out, 2, r.first_bad_link);
    if (r.has_checksum_response) {
        const BlockChecksumResponse &c = r.checksum_response;
        std::string cr;
        put_uint(cr, 1, c.bytes_per_crc);
        put_uint(cr, 2, c.crc_per_block);
        put_bytes(cr, 3, c.md5);
        if (c.crc_type >= 0) put_uint(cr, 4, uint64_t(c.crc_type));
        put_bytes(out, 3, cr);
    }
    if (r.has_checksum_info) {
        std::string cs;
        put_uint(cs, 1, uint64_t(r.checksum_type));
        put_uint(cs, 2, r.bytes_per_checksum);
        std::string info;
        put_bytes(info, 1, cs);
        put_uint(info, 2, r.chunk_offset);
        put_bytes(out, 4, info);
    }
    if (!r.message.empty()) put_bytes(out, 5, r.message);
    return out;
}

bool decode_block_op_response(const void *proto, size_t n, BlockOpResponse &out) {
    Reader r(proto, n);
    bool have_status = false;
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 0) {
            out.status = int(r.varint());
            have_status = true;
        } else if (field == 2 && wt == 2) {
            out.first_bad_link = r.bytes();
        } else if (field == 3 && wt == 2) {
            const std::string cr = r.bytes();
            Reader c(cr.data(), cr.size());
            BlockChecksumResponse &o = out.checksum_response;
            int seen = 0;
            while (c.more()) {
                const uint64_t k2 = c.varint();
                const int f2 = int(k2 >> 3), w2 = int(k2 & 7);
                if (f2 == 1 && w2 == 0) o.bytes_per_crc = uint32_t(c.varint()), seen |= 1;
                else if (f2 == 2 && w2 == 0) o.crc_per_block = c.varint(), seen |= 2;
                else if (f2 == 3 && w2 == 2) o.md5 = c.bytes(), seen |= 4;
                else if (f2 == 4 && w2 == 0) o.crc_type = int(c.varint());
                else c.skip(w2);
            }
            if (!c.ok || seen != 7) return false;   // the three fields are required
            out.has_checksum_response = true;
        } else if (field == 4 && wt == 2) {
            const std::string info = r.bytes();
            Reader i(info.data(), info.size());
            while (i.more()) {
                const uint64_t k2 = i.varint();
                const int f2 = int(k2 >> 3), w2 = int(k2 & 7);
                if (f2 == 1 && w2 == 2) {
                    const std::string cs = i.bytes();
                    Reader c(cs.data(), cs.size());
                    while (c.more()) {
                        const uint64_t k3 = c.varint();
                        const int f3 = int(k3 >> 3), w3 = int(k3 & 7);
                        if (f3 == 1 && w3 == 0) out.checksum_type = int(c.varint());
                        else if (f3 == 2 && w3 == 0) out.bytes_per_checksum = uint32_t(c.varint());
                        else c.skip(w3);
                    }
                    if (!c.ok) return false;
                } else if (f2 == 2 && w2 == 0) {
                    out.chunk_offset = i.varint();
                } else {
                    i.skip(w2);
                }
            }
            if (!i.ok) return false;
            out.has_checksum_info = true;
        } else if (field == 5 && wt == 2) {
            out.message = r.bytes();
        } else {
            r.skip(wt);
        }
    }
    return r.ok && have_status;
}

static std::string encode_datanode(const DatanodeAddr &d) {
    std::string id;
    put_bytes(id, 1, d.ip_addr);
    put_bytes(id, 2, d.host_name);
    put_bytes(id, 3, d.uuid);
    put_uint(id, 4, d.xfer_port);
    put_uint(id, 5, d.info_port);
    put_uint(id, 6, d.ipc_port);
    std::string info;
    put_bytes(info, 1, id);
    put_bytes(info, 8, d.location);  // always set by the reference (DataTransferProtocolSender.cpp:89)
    return info;
}

static bool decode_datanode(const std::string &s, DatanodeAddr &d) {
    Reader r(s.data(), s.size());
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 2) {
            const std::string id = r.bytes();
            Reader i(id.data(), id.size());
            while (i.more()) {
                const uint64_t k2 = i.varint();
                const int f2 = int(k2 >> 3), w2 = int(k2 & 7);
                if (f2 == 1 && w2 == 2) d.ip_addr = i.bytes();
                else if (f2 == 2 && w2 == 2) d.host_name = i.bytes();
                else if (f2 == 3 && w2 == 2) d.uuid = i.bytes();
                else if (f2 == 4 && w2 == 0) d.xfer_port = uint32_t(i.varint());
                else if (f2 == 5 && w2 == 0) d.info_port = uint32_t(i.varint());
                else if (f2 == 6 && w2 == 0) d.ipc_port = uint32_t(i.varint());
                else i.skip(w2);
            }
            if (!i.ok) return false;
        } else if (field == 8 && wt == 2) {
            d.location = r.bytes();
        } else {
            r.skip(wt);
        }
    }
    return r.ok;
}

std::string encode_write_block(const WriteBlockRequest &w) {
    std::string client_header;
    put_bytes(client_header, 1, encode_base_header(w.block));
    put_bytes(client_header, 2, w.client_name);
    std::string op;
    put_bytes(op, 1, client_header);
    for (const DatanodeAddr &t : w.targets) put_bytes(op, 2, encode_datanode(t));
    put_uint(op, 4, uint64_t(w.stage));
    put_uint(op, 5, w.pipeline_size);
    put_uint(op, 6, w.min_bytes_rcvd);
    put_uint(op, 7, w.max_bytes_rcvd);
    put_uint(op, 8, w.latest_generation_stamp);
    std::string ck;
    put_uint(ck, 1, uint64_t(w.checksum_type));
    put_uint(ck, 2, w.bytes_per_checksum);
    put_bytes(op, 9, ck);
    return frame_op(kOpWriteBlock, op);
}

bool decode_write_block(const void *proto, size_t n, WriteBlockRequest &out) {
    Reader r(proto, n);
    int seen = 0;
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 2) {
            const std::string ch = r.bytes();
            Reader h(ch.data(), ch.size());
            while (h.more()) {
                const uint64_t k2 = h.varint();
                const int f2 = int(k2 >> 3), w2 = int(k2 & 7);
                if (f2 == 1 && w2 == 2) {
                    const std::string base = h.bytes();
                    Reader b(base.data(), base.size());
                    while (b.more()) {
                        const uint64_t k3 = b.varint();
                        const int f3 = int(k3 >> 3), w3 = int(k3 & 7);
                        if (f3 == 1 && w3 == 2) {
                            if (!decode_extended_block(b.bytes(), out.block)) return false;
                        } else {
                            b.skip(w3);
                        }
                    }
                    if (!b.ok) return false;
                } else if (f2 == 2 && w2 == 2) {
                    out.client_name = h.bytes();
                } else {
                    h.skip(w2);
                }
            }
            if (!h.ok) return false;
            seen |= 1;
        } else if (field == 2 && wt == 2) {
            DatanodeAddr d;
            if (!decode_datanode(r.bytes(), d)) return false;
            out.targets.push_back(d);
        } else if (field == 4 && wt == 0) {
            out.stage = int(r.varint()), seen |= 2;
        } else if (field == 5 && wt == 0) {
            out.pipeline_size = uint32_t(r.varint()), seen |= 4;
        } else if (field == 6 && wt == 0) {
            out.min_bytes_rcvd = r.varint(), seen |= 8;
        } else if (field == 7 && wt == 0) {
            out.max_bytes_rcvd = r.varint(), seen |= 16;
        } else if (field == 8 && wt == 0) {
            out.latest_generation_stamp = r.varint(), seen |= 32;
        } else if (field == 9 && wt == 2) {
            const std::string ck = r.bytes();
            Reader c(ck.data(), ck.size());
            while (c.more()) {
                const uint64_t k2 = c.varint();
                const int f2 = int(k2 >> 3), w2 = int(k2 & 7);
                if (f2 == 1 && w2 == 0) out.checksum_type = int(c.varint());
                else if (f2 == 2 && w2 == 0) out.bytes_per_checksum = uint32_t(c.varint());
                else c.skip(w2);
            }
            if (!c.ok) return false;
            seen |= 64;
        } else {
            r.skip(wt);
        }
    }
    return r.ok && seen == 127;  // every required field (datatransfer.proto:78-109)
}

std::string encode_pipeline_ack(const PipelineAck &a) {
    std::string out;
    put_uint(out, 1, (uint64_t(a.seqno) << 1) ^ uint64_t(a.seqno >> 63));  // sint64: zigzag
    for (int s : a.status) put_uint(out, 2, uint64_t(s));
    if (a.downstream_ack_time_nanos) put_uint(out, 3, a.downstream_ack_time_nanos);
    return out;
}

bool decode_pipeline_ack(const void *proto, size_t n, PipelineAck &out) {
    Reader r(proto, n);
    bool have_seqno = false;
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 0) {
            const uint64_t z = r.varint();
            out.seqno = int64_t(z >> 1) ^ -int64_t(z & 1);
            have_seqno = true;
        } else if (field == 2 && wt == 0) {
            out.status.push_back(int(r.varint()));
        } else if (field == 2 && wt == 2) {  // packed encoding is legal for a repeated enum
            const std::string packed = r.bytes();
            Reader p(packed.data(), packed.size());
            while (p.more()) out.status.push_back(int(p.varint()));
            if (!p.ok) return false;
        } else if (field == 3 && wt == 0) {
            out.downstream_ack_time_nanos = r.varint();
        } else {
            r.skip(wt);
        }
    }
    return r.ok && have_seqno;
}

std::string encode_client_read_status(int status) {
    std::string out;
    put_uint(out, 1, uint64_t(status));
    return out;
}

bool decode_client_read_status(const void *proto, size_t n, int &status) {
    Reader r(proto, n);
    bool have = false;
    while (r.more()) {
        const uint64_t key = r.varint();
        const int field = int(key >> 3), wt = int(key & 7);
        if (field == 1 && wt == 0) {
            status = int(r.varint());
            have = true;
        } else {
            r.skip(wt);
        }
    }
    return r.ok && have;
}

}  // namespace wire
}  // namespace hdfs3crc
