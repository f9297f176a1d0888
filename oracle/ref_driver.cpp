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

}  // extern "C"
