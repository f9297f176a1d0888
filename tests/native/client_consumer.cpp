// A C++ consumer of the client drop-ins (include/hdfs3_client.h) in the shape of the
// reference's own function tests (test/function/TestOutputStream.cpp, TestInputStream.cpp):
// FillBuffer data ("012345678\n", mock/TestUtil.h:44-53) written with 1 KiB packets
// (TestInputStream.cpp:62 / TestOutputStream.cpp:86 output.default.packetsize=1024), read
// back in 20 KiB + 1 batches and checked with CheckBuffer (TestInputStream.cpp:256-273).
//
// Round trip: hdfs3_output_* computes every CRC on the GPU; the packets it emits are
// checked against the oracle (test infrastructure, oracle/crc32c_oracle.c) and reassembled
// into blocks; loopback datanodes (tools/loopback, test infrastructure) then serve those
// blocks WITH the GPU-written CRC words, and hdfs3_input_* verifies them on the GPU again.
// Last, each block's OP_BLOCK_CHECKSUM digest from both replicas is compared with the
// digest of the held words and with a GPU recomputation from each replica's bytes.
//
//   client_consumer   -> exit 0 = every check passed (needs a gfx950 device)
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <map>
#include <vector>

#include "crc32c_oracle.h"
#include "hdfs3_client.h"
#include "hdfs3_crc.h"

// tools/loopback/loopback_datanode.cpp (libhdfs3_loopback.so)
extern "C" {
int hdfs3_loopback_start(int *port);
int hdfs3_loopback_add_block(int port, uint64_t block_id, const void *data, uint64_t len, const void *crc_be,
                             uint32_t bpc, int checksum_type);
int hdfs3_loopback_set_packet_bytes(int port, int n);
int hdfs3_loopback_stop(int port);
}

static int g_fail = 0;
#define CHECK(cond, ...)                                              \
    do {                                                              \
        if (!(cond)) {                                                \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                        \
            std::fprintf(stderr, "\n");                               \
            ++g_fail;                                                 \
        }                                                             \
    } while (0)

static void fill_buffer(uint8_t *p, size_t n, size_t offset) {
    static const char pat[] = "012345678\n";
    for (size_t i = 0; i < n; ++i) p[i] = uint8_t(pat[(offset + i) % 10]);
}
static bool check_buffer(const uint8_t *p, size_t n, size_t offset) {
    static const char pat[] = "012345678\n";
    for (size_t i = 0; i < n; ++i)
        if (p[i] != uint8_t(pat[(offset + i) % 10])) return false;
    return true;
}
static uint32_t be32(const uint8_t *p) { return uint32_t(p[0]) << 24 | p[1] << 16 | p[2] << 8 | p[3]; }

constexpr uint32_t kBpc = 512;
constexpr int64_t kBlock = 1 << 20;

struct Collected {
    std::map<int64_t, std::vector<uint8_t>> data, crc;  // per block index
    int64_t packets = 0, last_packets = 0, next_seqno = 0;
};

static int sink(void *user, const void *packet, size_t len, const hdfs3_packet_info *info) {
    Collected &c = *static_cast<Collected *>(user);
    const uint8_t *p = static_cast<const uint8_t *>(packet);
    const size_t nch = size_t(info->num_chunks), dl = size_t(info->data_len);
    CHECK(len == 31 + 4 * nch + dl, "packet length %zu", len);
    // PacketHeader: BE32 packetLen = dataLen + checksumLen + 4 (Packet.cpp:124-153)
    CHECK(be32(p) == dl + 4 * nch + 4, "packetLen field %u", be32(p));
    CHECK(info->seqno == c.next_seqno, "seqno %lld, want %lld", (long long)info->seqno, (long long)c.next_seqno);
    c.next_seqno = info->seqno + 1;
    const uint8_t *words = p + 31, *data = words + 4 * nch;
    std::vector<uint8_t> want(4 * nch);
    if (dl) oracle_compute_chunks(1, data, dl, kBpc, want.data());
    CHECK(std::memcmp(words, want.data(), want.size()) == 0, "packet %lld: GPU CRC words differ from the oracle",
          (long long)info->seqno);
    std::vector<uint8_t> &bd = c.data[info->block_index];
    std::vector<uint8_t> &bc = c.crc[info->block_index];
    ++c.packets;
    c.last_packets += info->last_packet_in_block ? 1 : 0;
    // the empty last packet of a block carries offsetInBlock = bytesWritten, which counts
    // whole chunks only (OutputStreamImpl.cpp:311-320, 523): it adds no data
    if (!dl) return 0;
    // a flushed partial chunk is re-sent by the next packet from its chunk start
    CHECK(info->offset_in_block % kBpc == 0 && size_t(info->offset_in_block) <= bd.size(),
          "offsetInBlock %lld with %zu bytes held", (long long)info->offset_in_block, bd.size());
    bd.resize(size_t(info->offset_in_block));
    bd.insert(bd.end(), data, data + dl);
    bc.resize(size_t(info->offset_in_block / kBpc) * 4);
    bc.insert(bc.end(), words, words + 4 * nch);
    return 0;
}

// WriteFile (TestInputStream.cpp:275-293): 64 KiB FillBuffer pieces from offset 0
static void write_file(Collected &c, int64_t size) {
    hdfs3_writer_opts o{0, kBpc, 1024, kBlock, 64};
    hdfs3_output_stream *s = nullptr;
    CHECK(hdfs3_output_open(&o, sink, &c, &s) == 0, "output_open: %s", hdfs3_crc_last_error());
    if (!s) return;
    std::vector<uint8_t> buf(64 * 1024);
    int64_t off = 0;
    int n = 0;
    while (off < size) {
        const int32_t b = int32_t(std::min<int64_t>(buf.size(), size - off));
        fill_buffer(buf.data(), size_t(b), size_t(off));
        CHECK(hdfs3_output_write(s, buf.data(), b) == b, "write at %lld", (long long)off);
        off += b;
        if (++n % 7 == 0) CHECK(hdfs3_output_flush(s) == 0, "flush");  // partial chunks re-sent
    }
    CHECK(hdfs3_output_tell(s) == size, "tell");
    CHECK(hdfs3_output_close(s) == 0, "close");
}

// CheckFileContent (TestInputStream.cpp:256-273): 20 KiB + 1 reads, CheckBuffer each
static void check_file_content(const std::vector<hdfs3_located_block> &lbs, int64_t len) {
    hdfs3_reader_opts ro{0, 1, 64, 10000};
    hdfs3_input_stream *in = nullptr;
    CHECK(hdfs3_input_open(lbs.data(), int(lbs.size()), "client_consumer", &ro, &in) == 0, "input_open: %s",
          hdfs3_crc_last_error());
    if (!in) return;
    std::vector<uint8_t> buf(20 * 1024 + 1);
    int64_t off = 0;
    while (off < len) {
        const int32_t want = int32_t(std::min<int64_t>(buf.size(), len - off));
        const int32_t got = hdfs3_input_read(in, buf.data(), want);
        CHECK(got > 0, "read at %lld returned %d (%s)", (long long)off, got, hdfs3_crc_last_error());
        if (got <= 0) break;
        CHECK(check_buffer(buf.data(), size_t(got), size_t(off)), "CheckBuffer at %lld", (long long)off);
        off += got;
    }
    CHECK(hdfs3_input_read(in, buf.data(), 10) == 0, "read at EOF");
    CHECK(hdfs3_input_close(in) == 0, "input_close");
}

int main() {
    // ---- write: 3 blocks and a ragged tail through hdfs3_output_* ------------------------
    const int64_t size = 3 * kBlock + 234;
    Collected c;
    write_file(c, size);
    CHECK(c.data.size() == 4, "%zu blocks written", c.data.size());
    CHECK(c.last_packets == 4, "%lld last packets", (long long)c.last_packets);
    int64_t total = 0;
    for (auto &kv : c.data) {
        CHECK(check_buffer(kv.second.data(), kv.second.size(), size_t(total)), "block %lld content",
              (long long)kv.first);
        CHECK(c.crc[kv.first].size() == 4 * ((kv.second.size() + kBpc - 1) / kBpc), "block %lld words",
              (long long)kv.first);
        total += int64_t(kv.second.size());
    }
    CHECK(total == size, "%lld bytes written", (long long)total);

    // ---- serve the blocks with their GPU-written words, 1 KiB packets --------------------
    int good = 0, bad = 0;
    CHECK(hdfs3_loopback_start(&good) == 0 && hdfs3_loopback_start(&bad) == 0, "loopback start");
    hdfs3_loopback_set_packet_bytes(good, 1024);
    hdfs3_loopback_set_packet_bytes(bad, 1024);
    std::vector<uint8_t> corrupt = c.data[1];
    corrupt[kBlock / 2 + 17] ^= 0x20;  // block 1 of the bad replica, mid-block
    std::vector<hdfs3_datanode> both = {{"127.0.0.1", bad}, {"127.0.0.1", good}};
    std::vector<hdfs3_datanode> only_bad = {{"127.0.0.1", bad}};
    std::vector<hdfs3_located_block> lbs, lbs_bad;
    int64_t off = 0;
    for (auto &kv : c.data) {
        const uint64_t id = 9000 + uint64_t(kv.first);
        const std::vector<uint8_t> &d = kv.first == 1 ? corrupt : kv.second;
        hdfs3_loopback_add_block(good, id, kv.second.data(), kv.second.size(), c.crc[kv.first].data(), kBpc, 2);
        hdfs3_loopback_add_block(bad, id, d.data(), d.size(), c.crc[kv.first].data(), kBpc, 2);
        hdfs3_block_id b{"BP-loopback", id, 1, kv.second.size()};
        lbs.push_back(hdfs3_located_block{b, off, both.data(), 2});
        lbs_bad.push_back(hdfs3_located_block{b, off, only_bad.data(), 1});
        off += int64_t(kv.second.size());
    }

    // ---- read: the whole file, the corrupt replica first -> one failover -----------------
    check_file_content(lbs, size);
    {
        hdfs3_reader_opts ro{0, 1, 64, 10000};
        hdfs3_input_stream *in = nullptr;
        CHECK(hdfs3_input_open(lbs.data(), int(lbs.size()), "client_consumer", &ro, &in) == 0, "open");
        std::vector<uint8_t> all(static_cast<size_t>(size));
        int64_t pos = 0;
        while (in && pos < size) {
            const int32_t got = hdfs3_input_read(in, all.data() + pos, int32_t(std::min<int64_t>(1 << 20, size - pos)));
            if (got <= 0) break;
            pos += got;
        }
        uint64_t failovers = 0, opened = 0;
        if (in) hdfs3_input_stats(in, &failovers, &opened);
        CHECK(pos == size && check_buffer(all.data(), all.size(), 0), "full read (%lld bytes)", (long long)pos);
        CHECK(failovers == 1, "failovers %llu", (unsigned long long)failovers);
        // pread (TestInputStream.cpp:605-611 CheckFileContentByPread) across a block boundary
        std::vector<uint8_t> pr(300000);
        const int64_t at = kBlock - 1000;
        CHECK(in && hdfs3_input_pread(in, at, pr.data(), int32_t(pr.size())) == int32_t(pr.size()), "pread");
        CHECK(check_buffer(pr.data(), pr.size(), size_t(at)), "pread content");
        // seek past EOF: -1 / EOVERFLOW (HdfsEndOfStream, Hdfs.cpp:276-277)
        errno = 0;
        CHECK(in && hdfs3_input_seek(in, size + 1) == -1 && errno == EOVERFLOW, "seek past EOF: errno %d", errno);
        if (in) hdfs3_input_close(in);
    }

    // ---- every replica bad: good bytes, then -1 / EIO -----------------------------------
    {
        hdfs3_reader_opts ro{0, 1, 64, 10000};
        hdfs3_input_stream *in = nullptr;
        CHECK(hdfs3_input_open(lbs_bad.data(), int(lbs_bad.size()), "client_consumer", &ro, &in) == 0, "open bad");
        std::vector<uint8_t> buf(1 << 16);
        int64_t pos = 0;
        int32_t got = 0;
        errno = 0;
        while (in && (got = hdfs3_input_read(in, buf.data(), int32_t(buf.size()))) > 0) {
            CHECK(check_buffer(buf.data(), size_t(got), size_t(pos)), "good bytes before the error at %lld",
                  (long long)pos);
            pos += got;
        }
        CHECK(got == -1 && errno == EIO, "all replicas bad: read %d errno %d", got, errno);
        CHECK(pos >= kBlock && pos <= kBlock + kBlock / 2 + 17, "error surfaced at %lld", (long long)pos);
        if (in) hdfs3_input_close(in);
    }

    // ---- block checksums (OP_BLOCK_CHECKSUM, "MD5 of CRC32") and the file checksum -------
    // Both replicas hold the same stored CRC words, so both datanodes answer the same
    // digest; recomputing the words from each replica's bytes on the GPU tells the corrupt
    // replica of block 1 apart.
    {
        hdfs3_crc_ctx *ctx = nullptr;
        CHECK(hdfs3_crc_ctx_create(0, &ctx) == 0, "ctx_create: %s", hdfs3_crc_last_error());
        std::vector<uint8_t> digests;
        for (auto &kv : c.data) {
            const uint64_t id = 9000 + uint64_t(kv.first);
            const uint64_t words = c.crc[kv.first].size() / 4;
            hdfs3_block_id b{"BP-loopback", id, 1, kv.second.size()};
            hdfs3_block_checksum_info gi{}, bi{};
            CHECK(hdfs3_block_checksum_remote("127.0.0.1", good, &b, 10000, &gi) == 0, "block checksum: %s",
                  hdfs3_crc_last_error());
            CHECK(hdfs3_block_checksum_remote("127.0.0.1", bad, &b, 10000, &bi) == 0, "block checksum (bad)");
            uint8_t held[16];
            CHECK(hdfs3_block_checksum_crcs(c.crc[kv.first].data(), words, held) == 0, "checksum of held words");
            CHECK(std::memcmp(gi.md5, held, 16) == 0 && std::memcmp(bi.md5, held, 16) == 0, "block %lld md5",
                  (long long)kv.first);
            CHECK(gi.bytes_per_crc == kBpc && gi.crc_per_block == words && gi.crc_type == 2, "block %lld fields",
                  (long long)kv.first);
            for (int replica = 0; replica < 2 && ctx; ++replica) {
                const std::vector<uint8_t> &d = replica == 1 && kv.first == 1 ? corrupt : kv.second;
                void *dd = nullptr;
                uint8_t md5[16];
                uint64_t n = 0;
                CHECK(hdfs3_dev_malloc(&dd, d.size()) == 0 && hdfs3_memcpy_h2d(ctx, dd, d.data(), d.size()) == 0,
                      "upload");
                CHECK(hdfs3_block_checksum_dev(ctx, dd, d.size(), kBpc, md5, &n) == 0 && n == words,
                      "block_checksum_dev: %s", hdfs3_crc_last_error());
                const bool differs = std::memcmp(md5, gi.md5, 16) != 0;
                CHECK(differs == (replica == 1 && kv.first == 1), "block %lld replica %d: GPU digest %s",
                      (long long)kv.first, replica, differs ? "differs" : "matches");
                hdfs3_dev_free(dd);
            }
            digests.insert(digests.end(), gi.md5, gi.md5 + 16);
        }
        uint8_t file_md5[16];
        CHECK(hdfs3_file_checksum_md5md5crc(digests.data(), digests.size() / 16, file_md5) == 0, "file checksum");
        if (ctx) hdfs3_crc_ctx_destroy(ctx);
    }

    hdfs3_loopback_stop(good);
    hdfs3_loopback_stop(bad);
    if (g_fail)
        std::printf("client_consumer FAILED (%d)\n", g_fail);
    else
        std::printf("client_consumer ok (%lld packets)\n", (long long)c.packets);
    return g_fail ? 1 : 0;
}
