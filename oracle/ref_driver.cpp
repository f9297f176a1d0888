/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Thin extern "C" driver around the reference's own HWCrc32c engine, compiled
 * by oracle/Makefile directly from /root/reference/src/common/HWCrc32c.cpp
 * (container only; no reference source is copied into this repo). Output goes
 * to oracle/_ref/ (git-ignored). Used to generate tests/golden/ fixtures and as
 * the "reference" CPU baseline in bench.py.
 *
 * SWCrc32c is NOT built: SWCrc32c.h includes the cmake-generated platform.h
 * (src/platform.h.in), so it is unbuildable here. IntelAsmCrc32c needs yasm
 * (src/CMakeLists.txt:35-45), absent from this image.
 */
#include "HWCrc32c.h"

#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <time.h>
#include <arpa/inet.h>

#include "remote_loop.h"

using Hdfs::Internal::HWCrc32c;

extern "C" {

int ref_hw_available(void) { return HWCrc32c::available() ? 1 : 0; }

/* reset + update + getValue, as TestChecksum.cpp:91-97 drives it */
uint32_t ref_hw_crc32c(const void *p, int len) {
    HWCrc32c cs;
    cs.reset();
    cs.update(p, len);
    return cs.getValue();
}

/* Streamed update over `n` pieces, as TestChecksum.cpp:103-110 */
uint32_t ref_hw_crc32c_pieces(const void *const *ptrs, const int *lens, int n) {
    HWCrc32c cs;
    cs.reset();
    for (int i = 0; i < n; ++i) cs.update(ptrs[i], lens[i]);
    return cs.getValue();
}

/* The RemoteBlockReader::verifyChecksum loop (RemoteBlockReader.cpp:306-326) /
 * LocalBlockReader::readAndVerify loop (LocalBlockReader.cpp:138-163) driving the
 * reference engine; returns first bad chunk or -1 instead of throwing. */
int64_t ref_hw_verify(const void *data, int64_t len, int bpc, const void *crc_be,
                      int check_short_tail) {
    HWCrc32c cs;
    const char *d = static_cast<const char *>(data);
    const char *c = static_cast<const char *>(crc_be);
    int64_t chunks = (len + bpc - 1) / bpc;
    int64_t remaining = len;
    for (int64_t i = 0; i < chunks; ++i) {
        int size = bpc < remaining ? bpc : static_cast<int>(remaining);
        remaining -= size;
        cs.reset();
        cs.update(d + i * bpc, size);
        uint32_t target;
        memcpy(&target, c + 4 * i, 4);
        target = ntohl(target);
        if (cs.getValue() != target && (size == bpc || check_short_tail)) return i;
    }
    return -1;
}

struct RefBenchArg {
    const char *data, *crc;
    int64_t len;
    int bpc, reps;
    int64_t chunk0, bad;
};

static void *ref_bench_thread(void *p) {
    RefBenchArg *a = static_cast<RefBenchArg *>(p);
    a->bad = -1;
    for (int r = 0; r < a->reps; ++r) {
        int64_t b = ref_hw_verify(a->data, a->len, a->bpc, a->crc, 0);
        if (b >= 0 && a->bad < 0) a->bad = a->chunk0 + b;
    }
    return nullptr;
}

double ref_hw_bench_verify(const void *data, int64_t len, int bpc, const void *crc_be,
                           int threads, int reps, int64_t *bad_out) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    int64_t chunks = (len + bpc - 1) / bpc;
    int64_t per = (chunks + threads - 1) / threads;
    pthread_t tid[256];
    RefBenchArg args[256];
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int nt = 0;
    for (int t = 0; t < threads; ++t) {
        int64_t c0 = t * per;
        if (c0 >= chunks) break;
        int64_t c1 = c0 + per < chunks ? c0 + per : chunks;
        int64_t off = c0 * bpc;
        int64_t end = c1 * bpc < len ? c1 * bpc : len;
        args[t] = RefBenchArg{static_cast<const char *>(data) + off,
                              static_cast<const char *>(crc_be) + 4 * c0, end - off, bpc, reps,
                              c0, -1};
        pthread_create(&tid[t], nullptr, ref_bench_thread, &args[t]);
        ++nt;
    }
    int64_t bad = -1;
    for (int t = 0; t < nt; ++t) {
        pthread_join(tid[t], nullptr);
        if (args[t].bad >= 0 && (bad < 0 || args[t].bad < bad)) bad = args[t].bad;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (bad_out) *bad_out = bad;
    return double(t1.tv_sec - t0.tv_sec) + 1e-9 * double(t1.tv_nsec - t0.tv_nsec);
}

static int64_t ref_loop_verify(void *, const void *data, int64_t len, int bpc, const void *crc_be) {
    return ref_hw_verify(data, len, bpc, crc_be, 0);
}

/* One block through RemoteBlockReader's receive -> verify -> copy loop (oracle/remote_loop.h)
 * with the reference's HWCrc32c: the config-5 CPU baseline (bench.py). */
int64_t ref_remote_read_block(int fd, void *out, int64_t cap, int bpc, int verify, int64_t *bad_packet) {
    return remote_loop_read_block(fd, out, cap, bpc, verify, bad_packet, ref_loop_verify, nullptr);
}

/* The reference's write loop on one thread, for bench.py's config-5 write line: OutputStreamImpl::
 * appendInternal's whole-chunk path (OutputStreamImpl.cpp:298-359: checksum->update over the chunk,
 * appendChunkToPacket = Packet::addChecksum + addData, Packet.cpp:73-100) with the reference HWCrc32c,
 * packets of computePacketChunkSize chunks (:161-170), sendPacket when a packet is full or the block ends,
 * and each block's empty last packet (Packet::getBuffer framing: 31-byte header, then the BE words, then
 * the data). Every packet goes to a sink that touches one byte per 64 B (tools/loopback's count sink).
 * len a multiple of bpc. Returns seconds; *packets / *wire_bytes: what reached the sink. */
double ref_write_packets(const void *data, int64_t len, int bpc, int packet_size, int64_t block_size,
                         uint64_t *packets, uint64_t *wire_bytes) {
    const int hdr = 31, with_sum = bpc + 4;
    int cpp = (packet_size - hdr + with_sum - 1) / with_sum;
    if (cpp < 1) cpp = 1;
    char *pkt = static_cast<char *>(malloc(size_t(hdr) + size_t(cpp) * size_t(with_sum)));
    if (!pkt) return -1.0;
    HWCrc32c cs;
    const char *d = static_cast<const char *>(data);
    uint64_t np = 0, nb = 0, touch = 0;
    int64_t seq = 0;
    auto sink = [&](const char *p, size_t n) {
        for (size_t i = 0; i < n; i += 64) touch += uint8_t(p[i]);
        ++np;
        nb += n;
    };
    auto header = [&](int64_t off, int32_t dlen, bool last) {  // PacketHeader::writeInBuffer, 31 bytes
        const int32_t plen = dlen + 4 * ((dlen + bpc - 1) / bpc) + 4;
        const uint32_t be = htonl(uint32_t(plen));
        memcpy(pkt, &be, 4);
        pkt[4] = 0;
        pkt[5] = 25;
        pkt[6] = 0x09;
        memcpy(pkt + 7, &off, 8);
        pkt[15] = 0x11;
        memcpy(pkt + 16, &seq, 8);
        pkt[24] = 0x18;
        pkt[25] = last ? 1 : 0;
        pkt[26] = 0x25;
        memcpy(pkt + 27, &dlen, 4);
        ++seq;
    };
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int64_t b0 = 0; b0 < len; b0 += block_size) {
        const int64_t bend = b0 + block_size < len ? b0 + block_size : len;
        for (int64_t p0 = b0; p0 < bend;) {
            int n = 0;
            char *sums = pkt + hdr;
            char *pdata = sums + 4 * cpp;  // Packet's layout: checksums before data (getBuffer moves them)
            for (; n < cpp && p0 + int64_t(n) * bpc < bend; ++n) {
                const char *c = d + p0 + int64_t(n) * bpc;
                cs.reset();
                cs.update(c, bpc);
                const uint32_t w = htonl(cs.getValue());
                memcpy(sums + 4 * n, &w, 4);
                memcpy(pdata + int64_t(n) * bpc, c, size_t(bpc));
            }
            header(p0 - b0, n * bpc, false);
            if (n < cpp) memmove(sums + 4 * n, pdata, size_t(n) * size_t(bpc));  // getBuffer: words next to data
            sink(pkt, size_t(hdr) + size_t(n) * size_t(with_sum));
            p0 += int64_t(n) * bpc;
        }
        header(bend - b0, 0, true);  // the block's empty last packet
        sink(pkt, size_t(hdr));
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(pkt);
    if (packets) *packets = np + (touch & 0);
    if (wire_bytes) *wire_bytes = nb;
    return double(t1.tv_sec - t0.tv_sec) + 1e-9 * double(t1.tv_nsec - t0.tv_nsec);
}

}  // extern "C"
