// A C++ consumer of the drop-in C-ABI (include/hdfs3_crc.h), written the way the
// INTEGRATION.md patches call it from libhdfs3: no Python, no torch, only the header, the
// library and plain host/device pointers. The oracle (oracle/crc32c_oracle.c, test
// infrastructure) is the checker.
//
//   abi_consumer nodevice   -> expects hdfs3_crc_ctx_create to fail with -ENODEV (CPU box)
//   abi_consumer            -> full run on a gfx950 device; exit 0 = every check passed
//
// Cases mirror the reference call sites:
//   RemoteBlockReader::verifyChecksum (RemoteBlockReader.cpp:306-326): host verify of a
//     64 KiB packet, short tail ignored; first bad chunk reported.
//   LocalBlockReader::readAndVerify (LocalBlockReader.cpp:138-163): short tail checked.
//   OutputStreamImpl::appendInternal (OutputStreamImpl.cpp:298-359): compute of BE words.
//   packet arena with odd offsets (wire layout [chunks x BE32][data], :240-245).
//   device-resident block verify + async result word.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hdfs3_crc.h"

#include "crc32c_oracle.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);             \
            std::fprintf(stderr, "\n");                    \
            ++g_fail;                                      \
        }                                                  \
    } while (0)

static std::vector<uint8_t> oracle_words(const std::vector<uint8_t> &d, size_t len, uint32_t bpc) {
    std::vector<uint8_t> w(4 * ((len + bpc - 1) / bpc));
    oracle_compute_chunks(1 /* HWCrc32c restatement */, d.data(), len, bpc, w.data());
    return w;
}

int main(int argc, char **argv) {
    CHECK(hdfs3_crc_abi_version() == HDFS3_CRC_ABI_VERSION, "abi version");
    hdfs3_crc_ctx *ctx = nullptr;
    const int rc = hdfs3_crc_ctx_create(0, &ctx);
    if (argc > 1 && std::strcmp(argv[1], "nodevice") == 0) {
        // no silent CPU fallback: the engine refuses to exist without a gfx950 device
        CHECK(rc == -ENODEV && ctx == nullptr, "ctx_create without a device returned %d", rc);
        hdfs3_crc_ctx *pooled = nullptr;
        const int rc2 = hdfs3_crc_ctx_acquire(0, &pooled);
        CHECK(rc2 == -ENODEV && pooled == nullptr, "ctx_acquire without a device returned %d", rc2);
        CHECK(std::strlen(hdfs3_crc_last_error()) > 0, "no error message");
        std::printf(g_fail ? "abi_consumer nodevice FAILED\n" : "abi_consumer nodevice ok\n");
        return g_fail ? 1 : 0;
    }
    if (rc != 0) {
        std::fprintf(stderr, "ctx_create: %d %s\n", rc, hdfs3_crc_last_error());
        return 2;
    }

    // --- one 64 KiB packet, host API (RemoteBlockReader / OutputStreamImpl) ---------------
    const uint32_t bpc = 512;
    std::vector<uint8_t> pkt(65536);
    oracle_fill_splitmix(pkt.data(), pkt.size(), 0x5EED);
    std::vector<uint8_t> want = oracle_words(pkt, pkt.size(), bpc);
    std::vector<uint8_t> got(want.size());
    CHECK(hdfs3_crc32c_compute(ctx, pkt.data(), pkt.size(), bpc, got.data()) == 0, "compute: %s",
          hdfs3_crc_last_error());
    CHECK(got == want, "compute words differ from the oracle");
    int64_t bad = -2;
    CHECK(hdfs3_crc32c_verify(ctx, pkt.data(), pkt.size(), bpc, want.data(), 0, &bad) == 0 && bad == -1,
          "clean packet reported %lld", (long long)bad);
    for (int64_t k : {0, 77, 127}) {
        std::vector<uint8_t> flip = pkt;
        flip[k * bpc + 100] ^= 0x10;
        CHECK(hdfs3_crc32c_verify(ctx, flip.data(), flip.size(), bpc, want.data(), 0, &bad) == 0 && bad == k,
              "flip in chunk %lld reported %lld", (long long)k, (long long)bad);
    }

    // --- short tail: remote ignores a tail mismatch, local checks it ----------------------
    const size_t tail_len = 65536 - 100;
    std::vector<uint8_t> tw = oracle_words(pkt, tail_len, bpc);
    tw[tw.size() - 1] ^= 1;  // corrupt the stored word of the short tail chunk
    CHECK(hdfs3_crc32c_verify(ctx, pkt.data(), tail_len, bpc, tw.data(), 0, &bad) == 0 && bad == -1,
          "remote semantics flagged the short tail (%lld)", (long long)bad);
    CHECK(hdfs3_crc32c_verify(ctx, pkt.data(), tail_len, bpc, tw.data(), 1, &bad) == 0 &&
              bad == int64_t(tw.size() / 4 - 1),
          "local semantics missed the short tail (%lld)", (long long)bad);

    // --- packet arena in wire layout, odd offsets -----------------------------------------
    std::vector<uint8_t> arena(3 * (66048 + 7));
    std::vector<hdfs3_pkt_desc> pk(3);
    size_t off = 1;  // odd on purpose
    for (int p = 0; p < 3; ++p) {
        const uint32_t dl = p == 2 ? 65536 - 1000 : 65536;
        const size_t nch = (dl + bpc - 1) / bpc;
        std::vector<uint8_t> d(dl);
        oracle_fill_splitmix(d.data(), dl, 100 + p);
        std::vector<uint8_t> w = oracle_words(d, dl, bpc);
        std::memcpy(&arena[off], w.data(), 4 * nch);
        std::memcpy(&arena[off + 4 * nch], d.data(), dl);
        pk[p] = hdfs3_pkt_desc{off + 4 * nch, off, dl, 0};
        off += 4 * nch + dl + 3;
    }
    int64_t bp = -2, bc = -2;
    CHECK(hdfs3_crc32c_verify_packets(ctx, arena.data(), off, pk.data(), pk.size(), bpc, 0, &bp, &bc) == 0 &&
              bp == -1 && bc == -1,
          "clean packet arena reported (%lld, %lld)", (long long)bp, (long long)bc);
    arena[pk[1].data_off + 40 * bpc + 3] ^= 0x80;
    CHECK(hdfs3_crc32c_verify_packets(ctx, arena.data(), off, pk.data(), pk.size(), bpc, 0, &bp, &bc) == 0 &&
              bp == 1 && bc == 40,
          "packet flip reported (%lld, %lld)", (long long)bp, (long long)bc);

    // --- device-resident block + async result word ----------------------------------------
    const size_t blen = (8u << 20) + 300;
    std::vector<uint8_t> blk(blen);
    oracle_fill_splitmix(blk.data(), blen, 0xB10C);
    std::vector<uint8_t> bw = oracle_words(blk, blen, bpc);
    void *d_blk = nullptr, *d_crc = nullptr, *d_res = nullptr;
    CHECK(hdfs3_dev_malloc(&d_blk, blen) == 0 && hdfs3_dev_malloc(&d_crc, bw.size()) == 0 &&
              hdfs3_dev_malloc(&d_res, 8) == 0,
          "dev_malloc");
    CHECK(hdfs3_memcpy_h2d(ctx, d_blk, blk.data(), blen) == 0, "h2d");
    CHECK(hdfs3_crc32c_compute_dev(ctx, d_blk, blen, bpc, d_crc) == 0, "compute_dev");
    std::vector<uint8_t> dw(bw.size());
    CHECK(hdfs3_memcpy_d2h(ctx, dw.data(), d_crc, dw.size()) == 0 && dw == bw, "device words differ");
    CHECK(hdfs3_memset_dev(ctx, d_res, 0, 8) == 0, "memset");
    CHECK(hdfs3_crc32c_verify_dev_async(ctx, d_blk, blen, bpc, d_crc, 1, static_cast<uint64_t *>(d_res)) == 0,
          "verify_dev_async");
    uint64_t word = 1;
    CHECK(hdfs3_crc_ctx_synchronize(ctx) == 0 && hdfs3_memcpy_d2h(ctx, &word, d_res, 8) == 0, "result d2h");
    CHECK(hdfs3_crc_decode_result(word) == -1, "clean block decoded %lld", (long long)hdfs3_crc_decode_result(word));
    const uint8_t x = blk[12345 * bpc + 7] ^ 2;
    CHECK(hdfs3_memcpy_h2d(ctx, static_cast<uint8_t *>(d_blk) + 12345 * bpc + 7, &x, 1) == 0, "flip h2d");
    CHECK(hdfs3_crc32c_verify_dev(ctx, d_blk, blen, bpc, d_crc, 1, &bad) == 0 && bad == 12345,
          "device flip reported %lld", (long long)bad);
    // overlapped launches (HDFS3_LAUNCH_OVERLAP_PREVIOUS): a barriered first verify after the
    // memset, then chained ones; every result word still holds its own launch's answer
    void *d_res4 = nullptr;
    CHECK(hdfs3_dev_malloc(&d_res4, 32) == 0 && hdfs3_memset_dev(ctx, d_res4, 0, 32) == 0, "res4");
    for (int i = 0; i < 4; ++i)
        CHECK(hdfs3_crc32c_verify_dev_async_ex(ctx, d_blk, blen, bpc, d_crc, 1, static_cast<uint64_t *>(d_res4) + i,
                                               i ? HDFS3_LAUNCH_OVERLAP_PREVIOUS : 0) == 0,
              "verify_dev_async_ex %d", i);
    uint64_t words[4] = {0, 0, 0, 0};
    CHECK(hdfs3_crc_ctx_synchronize(ctx) == 0 && hdfs3_memcpy_d2h(ctx, words, d_res4, 32) == 0, "res4 d2h");
    for (int i = 0; i < 4; ++i)
        CHECK(hdfs3_crc_decode_result(words[i]) == 12345, "chained launch %d decoded %lld", i,
              (long long)hdfs3_crc_decode_result(words[i]));
    CHECK(hdfs3_crc32c_verify_dev_async_ex(ctx, d_blk, blen, bpc, d_crc, 1, static_cast<uint64_t *>(d_res4), 8u) ==
              -EINVAL,
          "unknown launch flag accepted");
    hdfs3_dev_free(d_res4);
    hdfs3_dev_free(d_blk);
    hdfs3_dev_free(d_crc);
    hdfs3_dev_free(d_res);

    // --- errors: negative errno, message, never a throw ------------------------------------
    CHECK(hdfs3_crc32c_verify(ctx, pkt.data(), pkt.size(), 0, want.data(), 0, &bad) == -EINVAL,
          "bpc 0 accepted");
    CHECK(std::strlen(hdfs3_crc_last_error()) > 0, "no message for EINVAL");
    CHECK(hdfs3_crc32c_verify(nullptr, pkt.data(), pkt.size(), bpc, want.data(), 0, &bad) == -EINVAL,
          "null ctx accepted");
    CHECK(hdfs3_crc_ctx_get_checksum_type(ctx) == HDFS3_CHECKSUM_TYPE_CRC32C, "default type");
    CHECK(hdfs3_crc_ctx_kernel_launches(ctx) > 0, "no kernel launched");

    // pooled contexts: a released context comes back on the next acquire, and works
    hdfs3_crc_ctx *p1 = nullptr, *p2 = nullptr;
    CHECK(hdfs3_crc_ctx_acquire(0, &p1) == 0 && p1, "acquire");
    hdfs3_crc_ctx_release(p1);
    CHECK(hdfs3_crc_ctx_acquire(0, &p2) == 0 && p2 == p1, "released context not reused");
    CHECK(hdfs3_crc32c_compute(p2, pkt.data(), pkt.size(), bpc, got.data()) == 0 && got == want, "pooled compute");
    hdfs3_crc_ctx_release(p2);

    hdfs3_crc_ctx_destroy(ctx);
    std::printf(g_fail ? "abi_consumer FAILED (%d)\n" : "abi_consumer ok\n", g_fail);
    return g_fail ? 1 : 0;
}
