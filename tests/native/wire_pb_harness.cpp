// Test infrastructure: a flat C interface over the product's wire codec
// (libhdfs3_amd/csrc/client/wire.cpp) so tests/test_wire_protobuf.py can check it against bytes
// produced and parsed by google.protobuf over the reference schema (tests/golden/proto_vectors.json).
//
// Messages are exchanged as text records, one `key=value` per line: integers in decimal, strings
// as `h:<hex>`; repeated keys repeat in order; write-block targets are `t<i>.<field>`.
//   long wh_encode(msg, kv, out, cap)  -> bytes written (the framed request for the ops, the
//                                         31-byte header for packet_header, the proto otherwise)
//   long wh_decode(msg, in, n, kv, cap) -> length of the record, -1 if the decoder rejected the
//                                         input, -2 if the record does not fit
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "client/wire.h"

using namespace hdfs3crc::wire;

namespace {

std::string hex(const std::string &s) {
    static const char *d = "0123456789abcdef";
    std::string o = "h:";
    for (unsigned char c : s) {
        o.push_back(d[c >> 4]);
        o.push_back(d[c & 15]);
    }
    return o;
}

std::string unhex(const std::string &v) {
    std::string o;
    if (v.compare(0, 2, "h:") != 0) return o;
    for (size_t i = 2; i + 1 < v.size(); i += 2) o.push_back(char(std::strtoul(v.substr(i, 2).c_str(), nullptr, 16)));
    return o;
}

struct Kv {
    std::multimap<std::string, std::string> m;
    std::vector<std::pair<std::string, std::string>> order;
    explicit Kv(const char *text) {
        const char *p = text;
        while (*p) {
            const char *nl = std::strchr(p, '\n');
            std::string line = nl ? std::string(p, nl) : std::string(p);
            const size_t eq = line.find('=');
            if (eq != std::string::npos) {
                m.emplace(line.substr(0, eq), line.substr(eq + 1));
                order.emplace_back(line.substr(0, eq), line.substr(eq + 1));
            }
            if (!nl) break;
            p = nl + 1;
        }
    }
    bool has(const std::string &k) const { return m.count(k) != 0; }
    std::string s(const std::string &k) const {
        auto it = m.find(k);
        return it == m.end() ? std::string() : unhex(it->second);
    }
    uint64_t u(const std::string &k, uint64_t def = 0) const {
        auto it = m.find(k);
        return it == m.end() ? def : std::strtoull(it->second.c_str(), nullptr, 10);
    }
    int64_t i(const std::string &k, int64_t def = 0) const {
        auto it = m.find(k);
        return it == m.end() ? def : std::strtoll(it->second.c_str(), nullptr, 10);
    }
    std::vector<std::string> all(const std::string &k) const {
        std::vector<std::string> v;
        for (const auto &kv : order)
            if (kv.first == k) v.push_back(kv.second);
        return v;
    }
};

struct Out {
    std::string t;
    void u(const char *k, uint64_t v) { t += std::string(k) + "=" + std::to_string(v) + "\n"; }
    void i(const char *k, int64_t v) { t += std::string(k) + "=" + std::to_string(v) + "\n"; }
    void s(const char *k, const std::string &v) { t += std::string(k) + "=" + hex(v) + "\n"; }
};

ExtendedBlock block_of(const Kv &kv) {
    ExtendedBlock b;
    b.pool_id = kv.s("pool");
    b.block_id = kv.u("block_id");
    b.generation_stamp = kv.u("gs");
    b.num_bytes = kv.u("num_bytes");
    return b;
}

void put_block(Out &o, const ExtendedBlock &b) {
    o.s("pool", b.pool_id);
    o.u("block_id", b.block_id);
    o.u("gs", b.generation_stamp);
    o.u("num_bytes", b.num_bytes);
}

long emit(const std::string &bytes, unsigned char *out, long cap) {
    if (long(bytes.size()) > cap) return -2;
    std::memcpy(out, bytes.data(), bytes.size());
    return long(bytes.size());
}

}  // namespace

extern "C" long wh_encode(const char *msg, const char *text, unsigned char *out, long cap) {
    const Kv kv(text);
    const std::string m(msg);
    if (m == "packet_header") {
        PacketHeader h;
        h.packet_len = int32_t(kv.i("packet_len"));
        h.offset_in_block = kv.i("offset");
        h.seqno = kv.i("seqno");
        h.last_packet_in_block = kv.u("last") != 0;
        h.data_len = int32_t(kv.i("data_len"));
        uint8_t b[kPacketHeaderSize];
        h.encode(b);
        return emit(std::string(reinterpret_cast<char *>(b), sizeof b), out, cap);
    }
    if (m == "read_block") {
        ReadBlockRequest r;
        r.block = block_of(kv);
        r.client_name = kv.s("client");
        r.offset = kv.u("offset");
        r.len = kv.u("len");
        r.send_checksums = kv.u("send_checksums", 1) != 0;
        return emit(encode_read_block(r), out, cap);
    }
    if (m == "block_checksum") return emit(encode_block_checksum(block_of(kv)), out, cap);
    if (m == "write_block") {
        WriteBlockRequest w;
        w.block = block_of(kv);
        w.client_name = kv.s("client");
        for (int t = 0; kv.has("t" + std::to_string(t) + ".ip"); ++t) {
            const std::string p = "t" + std::to_string(t) + ".";
            DatanodeAddr d;
            d.ip_addr = kv.s(p + "ip");
            d.host_name = kv.s(p + "host");
            d.uuid = kv.s(p + "uuid");
            d.xfer_port = uint32_t(kv.u(p + "xfer"));
            d.info_port = uint32_t(kv.u(p + "info"));
            d.ipc_port = uint32_t(kv.u(p + "ipc"));
            d.location = kv.s(p + "location");
            w.targets.push_back(d);
        }
        w.stage = int(kv.u("stage"));
        w.pipeline_size = uint32_t(kv.u("pipeline_size"));
        w.min_bytes_rcvd = kv.u("min_bytes");
        w.max_bytes_rcvd = kv.u("max_bytes");
        w.latest_generation_stamp = kv.u("latest_gs");
        w.checksum_type = int(kv.u("ck_type"));
        w.bytes_per_checksum = uint32_t(kv.u("bpc"));
        return emit(encode_write_block(w), out, cap);
    }
    if (m == "block_op_response") {
        BlockOpResponse r;
        r.status = int(kv.u("status"));
        r.first_bad_link = kv.s("first_bad_link");
        r.has_checksum_response = kv.has("cr.bpc");
        r.checksum_response.bytes_per_crc = uint32_t(kv.u("cr.bpc"));
        r.checksum_response.crc_per_block = kv.u("cr.crc_per_block");
        r.checksum_response.md5 = kv.s("cr.md5");
        r.checksum_response.crc_type = int(kv.i("cr.type", -1));
        r.has_checksum_info = kv.has("ci.type");
        r.checksum_type = int(kv.u("ci.type"));
        r.bytes_per_checksum = uint32_t(kv.u("ci.bpc"));
        r.chunk_offset = kv.u("ci.chunk_offset");
        r.message = kv.s("message");
        return emit(encode_block_op_response(r), out, cap);
    }
    if (m == "pipeline_ack") {
        PipelineAck a;
        a.seqno = kv.i("seqno");
        for (const std::string &v : kv.all("status")) a.status.push_back(int(std::strtol(v.c_str(), nullptr, 10)));
        a.downstream_ack_time_nanos = kv.u("downstream");
        return emit(encode_pipeline_ack(a), out, cap);
    }
    if (m == "client_read_status") return emit(encode_client_read_status(int(kv.u("status"))), out, cap);
    return -3;
}

extern "C" long wh_decode(const char *msg, const unsigned char *in, long n, char *text, long cap) {
    const std::string m(msg);
    Out o;
    bool ok = false;
    if (m == "packet_header") {
        PacketHeader h;
        ok = h.decode(in, size_t(n));
        o.i("packet_len", h.packet_len);
        o.i("offset", h.offset_in_block);
        o.i("seqno", h.seqno);
        o.u("last", h.last_packet_in_block);
        o.i("data_len", h.data_len);
        o.u("sync", h.sync_block);
    } else if (m == "read_block") {
        ReadBlockRequest r;
        ok = decode_read_block(in, size_t(n), r);
        put_block(o, r.block);
        o.s("client", r.client_name);
        o.u("offset", r.offset);
        o.u("len", r.len);
        o.u("send_checksums", r.send_checksums);
    } else if (m == "block_checksum") {
        ExtendedBlock b;
        ok = decode_block_checksum(in, size_t(n), b);
        put_block(o, b);
    } else if (m == "write_block") {
        WriteBlockRequest w;
        ok = decode_write_block(in, size_t(n), w);
        put_block(o, w.block);
        o.s("client", w.client_name);
        for (size_t t = 0; t < w.targets.size(); ++t) {
            const std::string p = "t" + std::to_string(t) + ".";
            const DatanodeAddr &d = w.targets[t];
            o.s((p + "ip").c_str(), d.ip_addr);
            o.s((p + "host").c_str(), d.host_name);
            o.s((p + "uuid").c_str(), d.uuid);
            o.u((p + "xfer").c_str(), d.xfer_port);
            o.u((p + "info").c_str(), d.info_port);
            o.u((p + "ipc").c_str(), d.ipc_port);
            o.s((p + "location").c_str(), d.location);
        }
        o.u("stage", uint64_t(w.stage));
        o.u("pipeline_size", w.pipeline_size);
        o.u("min_bytes", w.min_bytes_rcvd);
        o.u("max_bytes", w.max_bytes_rcvd);
        o.u("latest_gs", w.latest_generation_stamp);
        o.u("ck_type", uint64_t(w.checksum_type));
        o.u("bpc", w.bytes_per_checksum);
    } else if (m == "block_op_response") {
        BlockOpResponse r;
        ok = decode_block_op_response(in, size_t(n), r);
        o.u("status", uint64_t(r.status));
        if (!r.first_bad_link.empty()) o.s("first_bad_link", r.first_bad_link);
        if (r.has_checksum_response) {
            o.u("cr.bpc", r.checksum_response.bytes_per_crc);
            o.u("cr.crc_per_block", r.checksum_response.crc_per_block);
            o.s("cr.md5", r.checksum_response.md5);
            if (r.checksum_response.crc_type >= 0) o.i("cr.type", r.checksum_response.crc_type);
        }
        if (r.has_checksum_info) {
            o.u("ci.type", uint64_t(r.checksum_type));
            o.u("ci.bpc", r.bytes_per_checksum);
            o.u("ci.chunk_offset", r.chunk_offset);
        }
        if (!r.message.empty()) o.s("message", r.message);
    } else if (m == "pipeline_ack") {
        PipelineAck a;
        ok = decode_pipeline_ack(in, size_t(n), a);
        o.i("seqno", a.seqno);
        for (int s : a.status) o.i("status", s);
        o.u("downstream", a.downstream_ack_time_nanos);
    } else if (m == "client_read_status") {
        int s = -1;
        ok = decode_client_read_status(in, size_t(n), s);
        o.i("status", s);
    } else {
        return -3;
    }
    if (!ok) return -1;
    if (long(o.t.size()) + 1 > cap) return -2;
    std::memcpy(text, o.t.c_str(), o.t.size() + 1);
    return long(o.t.size());
}
