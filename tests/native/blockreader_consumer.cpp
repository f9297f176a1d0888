// integration/GpuRemoteBlockReader.h — a Hdfs::Internal::BlockReader compiled against the
// reference's own src/client/BlockReader.h and src/common/Exception.h, linked with the
// reference's src/common/Exception.cpp (its exception classes, built from source by the
// top-level Makefile into oracle/_ref/) — driven through the BlockReader interface exactly
// as InputStreamImpl::readOneBlock drives RemoteBlockReader (InputStreamImpl.cpp:616-708):
// read until 0, skip(), and a corrupt replica surfacing as Hdfs::ChecksumException (the
// exception readOneBlock catches to fail over, :682-688), a dead datanode as
// HdfsIOException. Words come from the oracle (test infrastructure). Needs a gfx950 GPU.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "GpuRemoteBlockReader.h"
#include "crc32c_oracle.h"

extern "C" {
int hdfs3_loopback_start(int *port);
int hdfs3_loopback_add_block(int port, uint64_t block_id, const void *data, uint64_t len, const void *crc_be,
                             uint32_t bpc, int checksum_type);
int hdfs3_loopback_stop(int port);
}

using Hdfs::Internal::BlockReader;
using Hdfs::Internal::GpuRemoteBlockReader;

static int g_fail = 0;
#define CHECK(c, ...)                                              \
    do {                                                           \
        if (!(c)) {                                                \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                     \
            std::fprintf(stderr, "\n");                            \
            ++g_fail;                                              \
        }                                                          \
    } while (0)

static std::unique_ptr<BlockReader> open_reader(int port, int64_t len, int64_t start = 0) {
    return std::unique_ptr<BlockReader>(new GpuRemoteBlockReader("127.0.0.1", port, "BP-loopback", 77, 1, len, start,
                                                                 len - start, "blockreader_consumer", true, 0, 10000));
}

int main() {
    const int64_t n = (4 << 20) + 777;
    const uint32_t bpc = 512;
    std::vector<uint8_t> data(n), crc(4 * ((n + bpc - 1) / bpc)), bad;
    oracle_fill_splitmix(data.data(), data.size(), 0x5EED);
    oracle_compute_chunks(1, data.data(), data.size(), bpc, crc.data());
    bad = data;
    const int64_t flip = 3 * 1000 * 1000 + 5;
    bad[flip] ^= 0x08;
    int good = 0, corrupt = 0;
    CHECK(hdfs3_loopback_start(&good) == 0 && hdfs3_loopback_start(&corrupt) == 0, "loopback");
    hdfs3_loopback_add_block(good, 77, data.data(), data.size(), crc.data(), bpc, 2);
    hdfs3_loopback_add_block(corrupt, 77, bad.data(), bad.size(), crc.data(), bpc, 2);

    std::vector<char> out(n);
    try {  // whole block through BlockReader::read
        auto r = open_reader(good, n);
        int64_t pos = 0;
        while (pos < n) pos += r->read(out.data() + pos, int32_t(std::min<int64_t>(1 << 20, n - pos)));
        CHECK(pos == n && std::memcmp(out.data(), data.data(), n) == 0, "clean read (%lld bytes)", (long long)pos);
        CHECK(r->available() == 0, "available at end");
        bool over = false;  // RemoteBlockReader::read past the range end throws HdfsIOException (:335-338)
        try {
            char c;
            r->read(&c, 1);
        } catch (const Hdfs::HdfsIOException &) {
            over = true;
        }
        CHECK(over, "read over the block end did not throw HdfsIOException");
    } catch (const Hdfs::HdfsException &e) {
        CHECK(false, "clean read threw: %s", e.what());
    }
    try {  // skip() then read: RemoteBlockReader::skip semantics
        auto r = open_reader(good, n);
        r->skip(100000);
        std::vector<char> rest(n - 100000);
        int64_t pos = 0;
        while (pos < int64_t(rest.size()))
            pos += r->read(rest.data() + pos, int32_t(std::min<int64_t>(1 << 20, rest.size() - pos)));
        CHECK(pos == int64_t(rest.size()) && std::memcmp(rest.data(), data.data() + 100000, rest.size()) == 0,
              "read after skip");
    } catch (const Hdfs::HdfsException &e) {
        CHECK(false, "skip threw: %s", e.what());
    }
    bool checksum_thrown = false;
    int64_t delivered = 0;
    try {  // corrupt replica: verified bytes, then ChecksumException (readOneBlock's failover cue)
        auto r = open_reader(corrupt, n);
        while (delivered < n)
            delivered += r->read(out.data() + delivered, int32_t(std::min<int64_t>(1 << 16, n - delivered)));
    } catch (const Hdfs::ChecksumException &e) {
        checksum_thrown = true;
    } catch (const Hdfs::HdfsException &e) {
        CHECK(false, "corrupt replica threw the wrong type: %s", e.what());
    }
    CHECK(checksum_thrown, "no ChecksumException from the corrupt replica");
    CHECK(delivered <= flip && std::memcmp(out.data(), data.data(), delivered) == 0, "bytes before the exception");
    bool io_thrown = false;
    try {  // nobody listening: HdfsIOException, not ChecksumException
        hdfs3_loopback_stop(corrupt);
        auto r = open_reader(corrupt, n);
    } catch (const Hdfs::ChecksumException &) {
        CHECK(false, "dead datanode reported as ChecksumException");
    } catch (const Hdfs::HdfsIOException &) {
        io_thrown = true;
    }
    CHECK(io_thrown, "no HdfsIOException from a dead datanode");
    hdfs3_loopback_stop(good);
    std::printf(g_fail ? "blockreader_consumer FAILED (%d)\n" : "blockreader_consumer ok\n", g_fail);
    return g_fail ? 1 : 0;
}
