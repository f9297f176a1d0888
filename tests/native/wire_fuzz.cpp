// TEST INFRASTRUCTURE — host-only sanitizer run of the wire codec the block reader uses on
// bytes that come from the network (libhdfs3_amd/csrc/client/wire.cpp). Built with
// -fsanitize=address,undefined by tests/test_wire_sanitized.py and run on the CPU:
//   1. encode -> decode round trips of random field values (identity)
//   2. random and mutated byte strings into every decoder (no crash / no UB; any result)
//   3. the PacketHeader sanity rules of PacketHeader.cpp:72-86 on random headers
// Deterministic (fixed seeds); exits non-zero on the first failed check.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "client/wire.h"

using namespace hdfs3crc::wire;

#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                             \
        }                                                             \
    } while (0)

static std::string rand_bytes(std::mt19937_64 &g, size_t n) {
    std::string s(n, '\0');
    for (auto &c : s) c = char(g() & 0xFF);
    return s;
}

static void mutate(std::mt19937_64 &g, std::string &s) {
    if (s.empty()) return;
    switch (g() % 4) {
    case 0: s[g() % s.size()] ^= char(1u << (g() % 8)); break;          // bit flip
    case 1: s.resize(g() % s.size()); break;                             // truncate
    case 2: s.insert(g() % (s.size() + 1), rand_bytes(g, 1 + g() % 8)); break;
    default: s[g() % s.size()] = char(0xFF); break;                      // varint poison
    }
}

int main(int argc, char **argv) {
    const long iters = argc > 1 ? std::atol(argv[1]) : 200000;
    std::mt19937_64 g(0x5EED);
    for (long it = 0; it < iters; ++it) {
        // 1. round trips
        PacketHeader h;
        h.packet_len = int32_t(4 + g() % (1u << 30));  // decode rejects < 4 (PacketHeader.cpp:105-110)
        h.offset_in_block = int64_t(g());
        h.seqno = int64_t(g());
        h.last_packet_in_block = g() & 1;
        h.data_len = int32_t(g());
        uint8_t buf[kPacketHeaderSize];
        h.encode(buf);
        PacketHeader d;
        CHECK(d.decode(buf, sizeof(buf)));
        CHECK(d.packet_len == h.packet_len && d.offset_in_block == h.offset_in_block && d.seqno == h.seqno &&
              d.last_packet_in_block == h.last_packet_in_block && d.data_len == h.data_len);

        BlockOpResponse r;
        r.status = int(g() % 8);
        r.has_checksum_info = g() & 1;
        r.checksum_type = int(g() % 3);
        r.bytes_per_checksum = uint32_t(g());
        r.chunk_offset = g();
        r.message = rand_bytes(g, g() % 40);
        std::string enc = encode_block_op_response(r);
        BlockOpResponse rd;
        CHECK(decode_block_op_response(enc.data(), enc.size(), rd));
        CHECK(rd.status == r.status && rd.has_checksum_info == r.has_checksum_info && rd.message == r.message);
        if (r.has_checksum_info)
            CHECK(rd.checksum_type == r.checksum_type && rd.bytes_per_checksum == r.bytes_per_checksum &&
                  rd.chunk_offset == r.chunk_offset);

        ReadBlockRequest q;
        q.block.pool_id = rand_bytes(g, g() % 24);
        q.block.block_id = g();
        q.block.generation_stamp = g();
        q.block.num_bytes = g();
        q.client_name = rand_bytes(g, g() % 24);
        q.offset = g();
        q.len = g();
        std::string frame = encode_read_block(q);
        CHECK(frame.size() > 3 && rd_be16(reinterpret_cast<const uint8_t *>(frame.data())) == kDataTransferVersion &&
              uint8_t(frame[2]) == kOpReadBlock);
        // skip the varint length after the 3-byte head
        size_t i = 3;
        uint64_t len = 0;
        for (int shift = 0; i < frame.size(); shift += 7) {
            const uint8_t b = uint8_t(frame[i++]);
            len |= uint64_t(b & 0x7F) << shift;
            if (!(b & 0x80)) break;
        }
        CHECK(len == frame.size() - i);
        ReadBlockRequest qd;
        CHECK(decode_read_block(frame.data() + i, len, qd));
        CHECK(qd.block.pool_id == q.block.pool_id && qd.block.block_id == q.block.block_id &&
              qd.client_name == q.client_name && qd.offset == q.offset && qd.len == q.len);

        const int st = int(g() % 8);
        std::string cs = encode_client_read_status(st);
        int sd = -1;
        CHECK(decode_client_read_status(cs.data(), cs.size(), sd) && sd == st);

        // 2. hostile inputs: random bytes, and mutated valid encodings
        std::string junk = rand_bytes(g, g() % 64);
        PacketHeader hj;
        (void)hj.decode(reinterpret_cast<const uint8_t *>(junk.data()), junk.size());
        BlockOpResponse rj;
        (void)decode_block_op_response(junk.data(), junk.size(), rj);
        ReadBlockRequest qj;
        (void)decode_read_block(junk.data(), junk.size(), qj);
        int sj;
        (void)decode_client_read_status(junk.data(), junk.size(), sj);
        std::string m1 = enc, m2(reinterpret_cast<const char *>(buf), sizeof(buf)), m3 = frame.substr(i);
        mutate(g, m1);
        mutate(g, m2);
        mutate(g, m3);
        (void)decode_block_op_response(m1.data(), m1.size(), rj);
        (void)hj.decode(reinterpret_cast<const uint8_t *>(m2.data()), m2.size());
        (void)decode_read_block(m3.data(), m3.size(), qj);

        // 3. sanity rules
        const int64_t last = int64_t(g() % 5) - 1;
        PacketHeader s = h;
        s.seqno = last + 1 + int64_t(g() % 2);
        s.data_len = int32_t(g() % 3) - 1;
        s.last_packet_in_block = g() & 1;
        const bool want = !(s.data_len <= 0 && !s.last_packet_in_block) &&
                          !(s.last_packet_in_block && s.data_len != 0) && s.seqno == last + 1;
        CHECK(s.sanity_check(last) == want);
    }
    std::printf("wire fuzz ok: %ld iterations\n", iters);
    return 0;
}
