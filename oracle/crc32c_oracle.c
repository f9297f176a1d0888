/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see crc32c_oracle.h).
 *
 * From-scratch C restatement of libhdfs3's CRC32C engines and per-chunk
 * verify/compute loops. CRC32C = reflected CRC-32 with polynomial 0x1EDC6F41
 * (reflected 0x82F63B78), init 0xFFFFFFFF, xorout 0xFFFFFFFF
 * (src/common/SWCrc32c.h:35,77-83).
 */
#define _GNU_SOURCE
#include "crc32c_oracle.h"

#include <nmmintrin.h>
#include <wmmintrin.h>
#include <pthread.h>
#include <string.h>
#include <time.h>

#define CRC32C_POLY_REFLECTED 0x82F63B78u

/* ---- table engine (SWCrc32c.cpp:47-104) --------------------------------- */

static uint32_t g_table[256];
/* crc_pcl combine constants (crc_iscsi_v_pcl.asm:221-245 uses K_table :342).
 * g_k[n][0] shifts block 0 over 16n bytes, g_k[n][1] shifts block 1 over 8n. */
static uint32_t g_k[129][2];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* x^e mod P in the reflected 32-bit representation (bit 31 = x^0). */
static uint32_t xpow_mod(unsigned e) {
    uint32_t v = 0x80000000u;
    while (e--) v = (v >> 1) ^ ((v & 1u) ? CRC32C_POLY_REFLECTED : 0u);
    return v;
}

static void init_tables(void) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? CRC32C_POLY_REFLECTED : 0u);
        g_table[i] = c;
    }
    /* clmul of two reflected 32-bit words yields x*A*B as a 64-bit reflected
     * qword; crc32q(0, q) then multiplies by x^32, so shifting a state over
     * d bytes needs K = x^(8d-33) mod P. */
    for (unsigned n = 1; n <= 128; ++n) {
        g_k[n][0] = xpow_mod(128u * n - 33u);
        g_k[n][1] = xpow_mod(64u * n - 33u);
    }
}

static inline void ensure_init(void) { pthread_once(&g_once, init_tables); }

uint32_t oracle_crc32c_sw_update(uint32_t crc, const void *b, size_t len) {
    ensure_init();
    const unsigned char *p = (const unsigned char *)b;
    const unsigned char *e = p + len;
    while (p < e) crc = g_table[(crc ^ *p++) & 0xFFu] ^ (crc >> 8);
    return crc;
}

/* ---- SSE4.2 engine (HWCrc32c.cpp:116-186) -------------------------------- */

static inline uint32_t hw_tail(uint32_t crc, const unsigned char *b, int len) {
    /* HWCrc32c::updateInt64 (HWCrc32c.cpp:152-186): 1..7 bytes as u8/u16/u32 pieces */
    switch (len) {
    case 7: crc = _mm_crc32_u8(crc, *b++); /* fallthrough */
    case 6: { uint16_t v; memcpy(&v, b, 2); crc = _mm_crc32_u16(crc, v); b += 2; }
            /* fallthrough */
    case 4: { uint32_t v; memcpy(&v, b, 4); crc = _mm_crc32_u32(crc, v); } break;
    case 3: crc = _mm_crc32_u8(crc, *b++); /* fallthrough */
    case 2: { uint16_t v; memcpy(&v, b, 2); crc = _mm_crc32_u16(crc, v); } break;
    case 5: { uint32_t v; memcpy(&v, b, 4); crc = _mm_crc32_u32(crc, v); b += 4; }
            /* fallthrough */
    case 1: crc = _mm_crc32_u8(crc, *b); break;
    default: break;
    }
    return crc;
}

uint32_t oracle_crc32c_hw_update(uint32_t crc, const void *buf, size_t len_in) {
    const unsigned char *p = (const unsigned char *)buf;
    size_t len = len_in;
    size_t align = 8 - ((uintptr_t)p % 8);
    if (align == 8) align = 0;
    if (len < align) align = len;
    crc = hw_tail(crc, p, (int)align);
    p += align;
    len -= align;
    for (size_t i = len / 8; i > 0; --i) {
        uint64_t v;
        memcpy(&v, p, 8);
        crc = (uint32_t)_mm_crc32_u64(crc, v);
        p += 8;
    }
    return hw_tail(crc, p, (int)(len & 7));
}

/* ---- crc_pcl behaviour (crc_iscsi_v_pcl.asm:93-340) ---------------------- */

static inline uint64_t ld64(const unsigned char *p) { uint64_t v; memcpy(&v, p, 8); return v; }

/* One 3-stream pass over n qwords per stream (asm crc_array :202-219, combine :221-245). */
static inline uint32_t pcl_block(uint32_t crc0, const unsigned char *p, unsigned n) {
    const unsigned char *b0 = p, *b1 = p + 8u * n, *b2 = p + 16u * n;
    uint64_t c0 = crc0, c1 = 0, c2 = 0;
    for (unsigned i = 0; i + 1 < n; ++i) {
        c0 = _mm_crc32_u64(c0, ld64(b0 + 8u * i));
        c1 = _mm_crc32_u64(c1, ld64(b1 + 8u * i));
        c2 = _mm_crc32_u64(c2, ld64(b2 + 8u * i));
    }
    c0 = _mm_crc32_u64(c0, ld64(b0 + 8u * (n - 1)));
    c1 = _mm_crc32_u64(c1, ld64(b1 + 8u * (n - 1)));
    __m128i k = _mm_set_epi32(0, (int)g_k[n][1], 0, (int)g_k[n][0]);
    __m128i x0 = _mm_clmulepi64_si128(_mm_cvtsi64_si128((long long)c0), k, 0x00);
    __m128i x1 = _mm_clmulepi64_si128(_mm_cvtsi64_si128((long long)c1), k, 0x10);
    uint64_t t = (uint64_t)_mm_cvtsi128_si64(_mm_xor_si128(x0, x1));
    return (uint32_t)_mm_crc32_u64(c2, t ^ ld64(b2 + 8u * (n - 1)));
}

uint32_t oracle_crc32c_pcl_update(uint32_t crc, const void *buf, size_t len) {
    ensure_init();
    const unsigned char *p = (const unsigned char *)buf;
    /* 1) align to 8 bytes (asm :110-138); short unaligned buffers go by-1 */
    size_t mis = (size_t)(-(intptr_t)p) & 7u;
    if (mis) {
        if (len < 8) {
            while (len--) crc = _mm_crc32_u8(crc, *p++);
            return crc;
        }
        for (size_t i = 0; i < mis; ++i) crc = _mm_crc32_u8(crc, *p++);
        len -= mis;
    }
    /* 2) full 3x128-qword blocks, then one partial block if >= SMALL_SIZE (asm :140-197) */
    while (len >= 128u * 24u) {
        crc = pcl_block(crc, p, 128);
        p += 128u * 24u;
        len -= 128u * 24u;
    }
    if (len >= 200u) {
        unsigned n = (unsigned)(len / 24u);
        crc = pcl_block(crc, p, n);
        p += 24u * n;
        len -= 24u * n;
    }
    /* 3) small path: by-8 then by-1 (asm :258-313) */
    while (len >= 8) {
        crc = (uint32_t)_mm_crc32_u64(crc, ld64(p));
        p += 8;
        len -= 8;
    }
    while (len--) crc = _mm_crc32_u8(crc, *p++);
    return crc;
}

static inline uint32_t engine_update(int engine, uint32_t s, const void *p, size_t n) {
    switch (engine) {
    case 0: return oracle_crc32c_sw_update(s, p, n);
    case 1: return oracle_crc32c_hw_update(s, p, n);
    default: return oracle_crc32c_pcl_update(s, p, n);
    }
}

uint32_t oracle_crc32c(int engine, const void *p, size_t len) {
    return ~engine_update(engine, 0xFFFFFFFFu, p, len);
}

/* ---- per-chunk loops ------------------------------------------------------ */

static inline uint32_t rd_be32(const unsigned char *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline void wr_be32(unsigned char *p, uint32_t v) {
    p[0] = (unsigned char)(v >> 24); p[1] = (unsigned char)(v >> 16);
    p[2] = (unsigned char)(v >> 8);  p[3] = (unsigned char)v;
}

void oracle_compute_chunks(int engine, const void *data, size_t len, uint32_t bpc,
                           void *crc_be_out) {
    const unsigned char *d = (const unsigned char *)data;
    unsigned char *o = (unsigned char *)crc_be_out;
    size_t chunks = (len + bpc - 1) / bpc;
    for (size_t i = 0; i < chunks; ++i) {
        size_t off = i * bpc;
        size_t sz = len - off < bpc ? len - off : bpc;
        wr_be32(o + 4 * i, oracle_crc32c(engine, d + off, sz));
    }
}

int64_t oracle_verify_chunks(int engine, const void *data, size_t len, uint32_t bpc,
                             const void *crc_be, int check_short_tail) {
    const unsigned char *d = (const unsigned char *)data;
    const unsigned char *c = (const unsigned char *)crc_be;
    size_t chunks = (len + bpc - 1) / bpc;
    for (size_t i = 0; i < chunks; ++i) {
        size_t off = i * bpc;
        size_t sz = len - off < bpc ? len - off : bpc;
        uint32_t got = oracle_crc32c(engine, d + off, sz);
        if (got != rd_be32(c + 4 * i) && (sz == bpc || check_short_tail)) return (int64_t)i;
    }
    return -1;
}

/* ---- multi-threaded CPU baseline ------------------------------------------ */

typedef struct {
    int engine;
    const unsigned char *data, *crc;
    size_t len;
    uint32_t bpc;
    int reps;
    int64_t chunk0;
    int64_t bad;
} bench_arg;

static void *bench_thread(void *a_) {
    bench_arg *a = (bench_arg *)a_;
    a->bad = -1;
    for (int r = 0; r < a->reps; ++r) {
        int64_t b = oracle_verify_chunks(a->engine, a->data, a->len, a->bpc, a->crc, 0);
        if (b >= 0 && a->bad < 0) a->bad = a->chunk0 + b;
    }
    return NULL;
}

double oracle_bench_verify(int engine, const void *data, size_t len, uint32_t bpc,
                           const void *crc_be, int threads, int reps, int64_t *bad_out) {
    ensure_init();
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    size_t chunks = (len + bpc - 1) / bpc;
    size_t per = (chunks + threads - 1) / threads;
    pthread_t tid[256];
    bench_arg args[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int nt = 0;
    for (int t = 0; t < threads; ++t) {
        size_t c0 = (size_t)t * per;
        if (c0 >= chunks) break;
        size_t c1 = c0 + per < chunks ? c0 + per : chunks;
        size_t off = c0 * bpc;
        size_t end = c1 * bpc < len ? c1 * bpc : len;
        args[t] = (bench_arg){engine, (const unsigned char *)data + off,
                              (const unsigned char *)crc_be + 4 * c0, end - off, bpc, reps,
                              (int64_t)c0, -1};
        pthread_create(&tid[t], NULL, bench_thread, &args[t]);
        ++nt;
    }
    int64_t bad = -1;
    for (int t = 0; t < nt; ++t) {
        pthread_join(tid[t], NULL);
        if (args[t].bad >= 0 && (bad < 0 || args[t].bad < bad)) bad = args[t].bad;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (bad_out) *bad_out = bad;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- deterministic data ---------------------------------------------------- */

void oracle_fill_splitmix(void *dst, size_t len, uint64_t seed) {
    unsigned char *o = (unsigned char *)dst;
    for (size_t i = 0; i * 8 < len; ++i) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        size_t n = len - i * 8 < 8 ? len - i * 8 : 8;
        memcpy(o + i * 8, &z, n);
    }
}

/* ---- CHECKSUM_CRC32 (boost::crc_32_type behind Crc32.h:41-75) --------------------------
 * Bit-serial restatement of the published algorithm (reflected, poly 0xEDB88320): slow on
 * purpose — an independent formulation from the GPU's slice tables. */
uint32_t oracle_crc32_update(uint32_t state, const void *p, size_t len) {
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < len; ++i) {
        state ^= b[i];
        for (int k = 0; k < 8; ++k) state = (state >> 1) ^ (0xEDB88320u & (0u - (state & 1u)));
    }
    return state;
}

void oracle_compute_chunks_crc32(const void *data, size_t len, uint32_t bpc, void *crc_be_out) {
    const unsigned char *d = (const unsigned char *)data;
    unsigned char *o = (unsigned char *)crc_be_out;
    size_t chunks = (len + bpc - 1) / bpc;
    for (size_t i = 0; i < chunks; ++i) {
        size_t off = i * bpc;
        size_t sz = len - off < bpc ? len - off : bpc;
        wr_be32(o + 4 * i, ~oracle_crc32_update(0xFFFFFFFFu, d + off, sz));
    }
}

/* ---- the reference's remote read loop (config-5 CPU baseline, oracle/remote_loop.h) ---- */

#include "remote_loop.h"

static int64_t loop_verify(void *user, const void *data, int64_t len, int bpc, const void *crc_be) {
    return oracle_verify_chunks(*(int *)user, data, (size_t)len, (uint32_t)bpc, crc_be, 0);
}

int64_t oracle_remote_read_block(int fd, int engine, void *out, int64_t cap, int bpc, int verify,
                                 int64_t *bad_packet) {
    ensure_init();
    return remote_loop_read_block(fd, out, cap, bpc, verify, bad_packet, loop_verify, &engine);
}
