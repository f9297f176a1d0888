// gfx950 (CDNA4) CRC32C kernels for libhdfs3's per-chunk checksum path: production
// launchers. The device code (kernels, design notes) is in crc32c_device.h; the kernel
// variants kept for A/B are in crc32c_experiments.hip.
#include "crc32c_wave.h"

namespace hdfs3crc {

#if HDFS3_LAB
int g_variant = 0;  // measurement knob (hdfs3x_set_variant); 0 = production choice
#endif

namespace {

template <int BPC, bool V>
hipError_t launch_r(const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                    hipStream_t s) {
    // Production path: the round kernel of crc32c_wave.h for bpc <= 4096, late prefetch, the solo
    // last step for overlapped launches up to 256 MiB (HDFS3_LAUNCH_OVERLAP_PREVIOUS: an AQL packet
    // without the barrier bit); the multi-round kernel above 4096. Non-zero variants select the designs kept
    // for in-process A/B (crc32c_experiments.hip, tools/ab.py).
#if HDFS3_LAB
    if (g_variant != 0) return launch_experiment(g_variant, a, V, tab, fold, grid_cap, s);
#endif
    if constexpr (BPC <= kRoundBytes) return launch_wave3<BPC, V, false, true>(a, tab, fold, grid_cap, s);
    return launch_r3<BPC, V, 1, true>(a, tab, fold, grid_cap, s);
}

template <int BPC>
hipError_t launch_rv(const ChunkLaunch &a, bool verify, const uint32_t *tab, const uint32_t *fold,
                     int grid_cap, hipStream_t s) {
    return verify ? launch_r<BPC, true>(a, tab, fold, grid_cap, s)
                  : launch_r<BPC, false>(a, tab, fold, grid_cap, s);
}

// packet streams at a constant pitch: the production round kernel's pitch walk
template <int BPC, bool V>
hipError_t launch_p(const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap, hipStream_t s) {
#if HDFS3_LAB
    if (g_variant == 115) return launch_wave3<BPC, V, true, true, kLabPrio>(a, tab, fold, grid_cap, s);
    if (g_variant == 117) return launch_wave3<BPC, V, true, true, kLabNoPrio>(a, tab, fold, grid_cap, s);
    // without the solo last step (production before round 4)
    if (g_variant == 124) return launch_wave3<BPC, V, true, false>(a, tab, fold, grid_cap, s);
    // 256-thread workgroups (4 waves each): small launches spread over 4x the CUs
    if (g_variant == 132) return launch_wave3<BPC, V, true, true, 0, 256>(a, tab, fold, grid_cap, s);
    if (g_variant == 134) return launch_wave3<BPC, V, true, true, 0, 512>(a, tab, fold, grid_cap, s);
    if (g_variant == 137) return launch_wave3<BPC, V, true, true, kLabWg1024>(a, tab, fold, grid_cap, s);
    // compute: each round's words stored at once instead of held (round 6, the writer's small batches)
    if (g_variant == 163) return launch_wave3<BPC, V, true, true, kLabNoHold>(a, tab, fold, grid_cap, s);
    // one round per wave for launches of <= 4096 units (round 6)
    if (g_variant == 162) return launch_wave3<BPC, V, true, true, kLabOneRound>(a, tab, fold, grid_cap, s);
#endif
    // the solo last step for overlapped launches up to 256 MiB, as the block walk (round 4): 128 MiB of
    // 64 KiB packets at the block reader's 66,048-byte pitch 22.53 -> 20.98 us overlapped against 20.97
    // for the same payload as one contiguous block (tools/pkt_ab.py, profiles/r04/r4c_pkt_ab*)
    return launch_wave3<BPC, V, true, true>(a, tab, fold, grid_cap, s);
}

template <int BPC>
hipError_t launch_pv(const ChunkLaunch &a, bool verify, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                     hipStream_t s) {
    return verify ? launch_p<BPC, true>(a, tab, fold, grid_cap, s) : launch_p<BPC, false>(a, tab, fold, grid_cap, s);
}


}  // namespace

bool packet_geom(uint64_t data_len, uint64_t last_len, uint64_t npk, uint32_t unit_bpc, PacketGeom *g) {
    if (npk == 0 || unit_bpc == 0 || unit_bpc > uint32_t(kRoundBytes) || last_len > data_len) return false;
    if (npk > 1 && (data_len == 0 || data_len % unit_bpc)) return false;  // only the last packet ends short
    PacketGeom r;
    r.pk_len = npk > 1 ? data_len : 0;
    r.upp = uint32_t(npk > 1 ? (data_len + kRoundBytes - 1) / kRoundBytes : 1);
    r.ptail = uint32_t(npk > 1 ? data_len - uint64_t(r.upp - 1) * kRoundBytes : kRoundBytes);
    const uint64_t lw = last_len / unit_bpc * unit_bpc;
    r.lunits = uint32_t((lw + kRoundBytes - 1) / kRoundBytes);
    r.ltail = r.lunits ? uint32_t(lw - uint64_t(r.lunits - 1) * kRoundBytes) : 0;
    const uint64_t units = (npk - 1) * uint64_t(r.upp) + r.lunits;
    if (units == 0 || units >= (uint64_t(1) << 31)) return false;
    // q = (u * magic) >> shift = u / upp for every u < 2^31: magic = ceil(2^(31 + l) / upp), l =
    // ceil(log2 upp), so magic < 2^32 and u * magic < 2^63
    uint32_t l = 0;
    while ((uint64_t(1) << l) < r.upp) ++l;
    r.shift = 31 + l;
    r.magic = uint32_t(((uint64_t(1) << r.shift) + r.upp - 1) / r.upp);
    *g = r;
    return true;
}

bool packet_stream_ok(uint64_t data_len, uint64_t last_len, uint64_t npk, uint32_t bpc, const void *data,
                      const void *crc, uint64_t pitch, PacketGeom *geom) {
    // bpc 512..4096: the round kernel's pitch walk, a packet's last round partial when its chunks
    // end inside one (round 6); R * 4096 (R >= 2): the walk's 4096-byte piece CRCs + the combine
    // (launch_stream_pieces, round 4), every packet but the last whole chunks
    const bool pieces = bpc > kRoundBytes && bpc % kRoundBytes == 0;
    if (bpc != 512 && bpc != 1024 && bpc != 2048 && bpc != 4096 && !pieces) return false;
    if (npk == 0 || data_len == 0 || last_len > data_len) return false;
    if (npk > 1 && pitch == 0) return false;
    if (npk >= (uint64_t(1) << 31)) return false;  // keys are (packet << 32) | chunk
    if ((reinterpret_cast<uintptr_t>(data) & 15u) || (reinterpret_cast<uintptr_t>(crc) & 3u) || (pitch & 15u))
        return false;
    if (pieces && npk > 1 && data_len % bpc) return false;
    return packet_geom(data_len, last_len, npk, pieces ? uint32_t(kRoundBytes) : bpc, geom);
}

hipError_t launch_strided_blocks(const DevSegment *h_seg, size_t n, uint32_t bpc, bool verify, int check_short_tail,
                                 unsigned long long *result, const uint32_t *d_tables, const uint32_t *d_fold,
                                 int grid_cap, hipStream_t stream, WordScratch *ws) {
#if HDFS3_LAB
    if (g_variant == 54) return hipErrorNotSupported;  // A/B: force the segmented kernel
#endif
    if (n < 2) return hipErrorNotSupported;
    const int64_t dp = h_seg[1].data - h_seg[0].data, cp = h_seg[1].crc - h_seg[0].crc;
    if (dp <= 0 || cp <= 0) return hipErrorNotSupported;
    for (size_t i = 0; i < n; ++i)
        if (h_seg[i].data != h_seg[0].data + int64_t(i) * dp || h_seg[i].crc != h_seg[0].crc + int64_t(i) * cp ||
            (i + 1 < n && h_seg[i].len != h_seg[0].len) || h_seg[i].len > h_seg[0].len)
            return hipErrorNotSupported;
    PacketGeom geom;
    if (!packet_stream_ok(h_seg[0].len, h_seg[n - 1].len, n, bpc, h_seg[0].data, h_seg[0].crc, uint64_t(dp),
                          &geom) ||
        (cp & 3))
        return hipErrorNotSupported;
    ChunkLaunch a{};
    a.data = h_seg[0].data;
    a.crc_be = h_seg[0].crc;
    a.out_be = h_seg[0].crc;
    a.bpc = bpc;
    a.result = result;
    a.check_short_tail = check_short_tail;
    a.pitch = uint64_t(dp);
    a.crc_pitch = uint64_t(cp);
    a.npk = n;
    a.geom = geom;
    a.last_len = uint32_t(h_seg[n - 1].len);
    return launch_packet_stream(a, verify, d_tables, d_fold, grid_cap, stream, ws);
}

namespace {

// packet p's `words` bytes (`last` for the last packet) from src + p * src_pitch to
// dst + p * dst_pitch: one wave per packet at a time, 64 consecutive words per store
__global__ __launch_bounds__(256) void crc32c_scatter_words_kernel(const uint8_t *__restrict__ src, uint8_t *dst,
                                                                   uint64_t src_pitch, uint64_t dst_pitch,
                                                                   uint64_t npk, uint32_t words, uint32_t last) {
    const uint64_t nwaves = uint64_t(gridDim.x) * 4;
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t p = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); p < npk; p += nwaves) {
        const uint32_t nw = (p + 1 == npk ? last : words) / 4;
        const uint32_t *s = reinterpret_cast<const uint32_t *>(src + p * src_pitch);
        uint32_t *d = reinterpret_cast<uint32_t *>(dst + p * dst_pitch);
        for (uint32_t i = lane; i < nw; i += 64) d[i] = s[i];
    }
}

hipError_t launch_stream_kernel(const ChunkLaunch &a, bool verify, const uint32_t *d_tables, const uint32_t *d_fold,
                                int grid_cap, hipStream_t stream) {
    switch (a.bpc) {
    case 512: return launch_pv<512>(a, verify, d_tables, d_fold, grid_cap, stream);
    case 1024: return launch_pv<1024>(a, verify, d_tables, d_fold, grid_cap, stream);
    case 2048: return launch_pv<2048>(a, verify, d_tables, d_fold, grid_cap, stream);
    case 4096: return launch_pv<4096>(a, verify, d_tables, d_fold, grid_cap, stream);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

// bpc = R * 4096 packet streams (defined with launch_pieces below)
hipError_t launch_stream_pieces(const ChunkLaunch &a, bool verify, const uint32_t *d_tables, const uint32_t *d_fold,
                                int grid_cap, hipStream_t stream, PieceScratch *ps);

void WordScratch::release() {
    if (d) (void)hipFree(d);
    if (used) (void)hipEventDestroy(used);
    *this = WordScratch();
}

hipError_t launch_packet_stream(const ChunkLaunch &a, bool verify, const uint32_t *d_tables, const uint32_t *d_fold,
                                int grid_cap, hipStream_t stream, WordScratch *ws, PieceScratch *pieces) {
#if HDFS3_LAB
    if (g_variant == 52 || g_variant == 53) return hipErrorNotSupported;  // A/B: force the segmented kernel
    if (g_variant == 55) ws = nullptr;  // A/B: words written in place (no dense scratch)
#endif
    if (a.bpc > kRoundBytes) {  // chunks of R whole rounds: pieces + combine, or the caller's fallback
        if (!pieces || a.bpc % kRoundBytes || (a.npk > 1 && a.geom.pk_len % a.bpc)) return hipErrorNotSupported;
        return launch_stream_pieces(a, verify, d_tables, d_fold, grid_cap, stream, pieces);
    }
    if (a.bpc != 512 && a.bpc != 1024 && a.bpc != 2048 && a.bpc != 4096) return hipErrorInvalidValue;
    const uint64_t cpitch = a.crc_pitch ? a.crc_pitch : a.pitch;
    const uint64_t wpp = a.geom.pk_len / a.bpc * 4;  // word bytes per packet
    if (!verify && ws && a.npk > 1 && cpitch > wpp && wpp <= kDenseWordsMaxRegion) {
        const uint64_t last = (uint64_t(a.last_len) + a.bpc - 1) / a.bpc * 4;
        const uint64_t need = (a.npk - 1) * wpp + last;
        if (need > ws->cap) {
            // the old scratch may still be read by a launch in flight (any stream)
            if (ws->used) {
                hipError_t e = hipEventSynchronize(ws->used);
                if (e != hipSuccess) return e;
            }
            if (ws->d) (void)hipFree(ws->d);
            ws->d = nullptr;
            ws->cap = 0;
            hipError_t e = hipMalloc(reinterpret_cast<void **>(&ws->d), need);
            if (e != hipSuccess) return e;
            ws->cap = need;
        }
        if (!ws->used) {
            hipError_t e = hipEventCreateWithFlags(&ws->used, hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        ChunkLaunch b = a;
        b.out_be = ws->d;
        b.crc_be = ws->d;
        b.crc_pitch = wpp;
        hipError_t e = launch_stream_kernel(b, false, d_tables, d_fold, grid_cap, stream);
        if (e != hipSuccess) return e;
        const uint64_t need_waves = a.npk, cap_waves = 4096;
        const int grid = int(((need_waves < cap_waves ? need_waves : cap_waves) + 3) / 4);
        hipLaunchKernelGGL(crc32c_scatter_words_kernel, dim3(grid), dim3(256), 0, stream, ws->d, a.out_be, wpp, cpitch,
                           a.npk, uint32_t(wpp), uint32_t(last));
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        return hipEventRecord(ws->used, stream);
    }
    return launch_stream_kernel(a, verify, d_tables, d_fold, grid_cap, stream);
}

constexpr uint64_t kPiecesMinBytes = uint64_t(256) << 20;

void PieceScratch::release() {
    for (int i = 0; i < 2; ++i) {
        if (d[i]) (void)hipFree(d[i]);
        if (used[i]) (void)hipEventDestroy(used[i]);
    }
    *this = PieceScratch();
}

namespace {

// Chunk c of R 4096-byte pieces from the pieces' CRCs y_i (standard init and final xor, BE words in
// `piece_be`): with A = the 4096-zero-byte advance (d_fold + kFoldAdvance4096) and crc0 the raw
// (init 0, no final xor) CRC, crc0(P_i) = y_i ^ K, K = A(~0) ^ ~0, and the chunk's state from init ~0
// is s = A(... A(A(~0) ^ crc0(P_0)) ...) ^ crc0(P_{R-1}); its CRC is ~s. One chunk per thread.
// cpp > 0 (packet streams, round 4): chunk k is chunk k % cpp of packet k / cpp, its word at
// crc + (k / cpp) * cpitch + 4 (k % cpp) and its key (packet << 32) | chunk; the pieces stay dense.
template <bool VERIFY>
__global__ __launch_bounds__(256) void crc32c_combine_pieces_kernel(const uint8_t *__restrict__ piece_be, uint64_t nchunks,
                                                                    uint32_t R, const uint32_t *__restrict__ g_fold,
                                                                    const uint8_t *crc_be, uint8_t *out_be,
                                                                    uint64_t chunk_base,
                                                                    unsigned long long *result, uint64_t cpp = 0,
                                                                    uint64_t cpitch = 0) {
    uint32_t col[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) col[i] = g_fold[kFoldAdvance4096 + i];
    const uint32_t K = gf2_apply4(col, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    const uint32_t *y = reinterpret_cast<const uint32_t *>(piece_be);
    for (uint64_t c = uint64_t(blockIdx.x) * 256 + threadIdx.x; c < nchunks; c += uint64_t(gridDim.x) * 256) {
        uint32_t st = 0xFFFFFFFFu;
        for (uint32_t i = 0; i < R; ++i) st = gf2_apply4(col, st) ^ __builtin_bswap32(y[c * R + i]) ^ K;
        const uint32_t v = ~st;
        uint64_t woff = 4 * c, key = chunk_base + c;
        if (cpp) {
            const uint64_t pk = c / cpp, ch = c % cpp;
            woff = pk * cpitch + 4 * ch;
            key = (pk << 32) | ch;
        }
        if constexpr (VERIFY) {
            if (__builtin_bswap32(*reinterpret_cast<const uint32_t *>(crc_be + woff)) != v)
                atomicMax(result, ~(unsigned long long)key);
        } else {
            *reinterpret_cast<uint32_t *>(out_be + woff) = __builtin_bswap32(v);
        }
    }
}

// Whole chunks of R = bpc / 4096 pieces: the round kernel's compute at bpc 4096 into the scratch,
// then the combine. The short tail chunk (if any) goes to the chunk-per-lane kernel.
// The next of the two piece buffers, at least `need` bytes, ordered after its previous reader.
hipError_t piece_buffer(PieceScratch *ps, uint64_t need, hipStream_t stream, unsigned *out) {
    const unsigned b = ps->next & 1u;
    if (need > ps->cap[b]) {
        if (ps->used[b]) {  // the buffer may still be read by a combine in flight
            hipError_t e = hipEventSynchronize(ps->used[b]);
            if (e != hipSuccess) return e;
        }
        if (ps->d[b]) (void)hipFree(ps->d[b]);
        ps->d[b] = nullptr;
        ps->cap[b] = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void **>(&ps->d[b]), need);
        if (e != hipSuccess) return e;
        ps->cap[b] = need;
    }
    if (!ps->used[b]) {
        hipError_t e = hipEventCreateWithFlags(&ps->used[b], hipEventDisableTiming);
        if (e != hipSuccess) return e;
    } else if (ps->on[b] != stream) {
        // the last reader of this buffer ran on another stream (the ctx's stream was switched):
        // order this launch after it; on one stream the launch order already does
        hipError_t e = hipStreamWaitEvent(stream, ps->used[b], 0);
        if (e != hipSuccess) return e;
    }
    ps->on[b] = stream;
    ps->next = b + 1;
    *out = b;
    return hipSuccess;
}

hipError_t launch_pieces(const ChunkLaunch &a, bool verify, const uint32_t *d_tables, const uint32_t *d_fold,
                         int grid_cap, hipStream_t stream, PieceScratch *ps) {
    const uint32_t R = a.bpc / kRoundBytes;
    const uint64_t nfull = a.len / a.bpc;
    unsigned b = 0;
    if (hipError_t e = piece_buffer(ps, nfull * R * 4, stream, &b); e != hipSuccess) return e;
    ChunkLaunch p = a;  // the pieces: a compute at bpc 4096 over the whole chunks
    p.len = nfull * a.bpc;
    p.bpc = kRoundBytes;
    p.out_be = ps->d[b];
    p.crc_be = nullptr;
    p.chunk_base = 0;
    hipError_t e = launch_wave3<kRoundBytes, false, false, true>(p, d_tables, d_fold, grid_cap, stream);
    if (e != hipSuccess) return e;
    const uint64_t blocks = (nfull + 255) / 256;
    const int grid = int(blocks < 1024 ? blocks : 1024);
    if (verify)
        hipLaunchKernelGGL(crc32c_combine_pieces_kernel<true>, dim3(grid), dim3(256), 0, stream, ps->d[b], nfull, R,
                           d_fold, a.crc_be, nullptr, a.chunk_base, a.result);
    else
        hipLaunchKernelGGL(crc32c_combine_pieces_kernel<false>, dim3(grid), dim3(256), 0, stream, ps->d[b], nfull, R,
                           d_fold, nullptr, a.out_be, a.chunk_base, a.result);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipEventRecord(ps->used[b], stream);
    if (e != hipSuccess) return e;
    const uint64_t tail = a.len - nfull * a.bpc;
    if (tail == 0) return hipSuccess;
    ChunkLaunch t = a;  // the short tail chunk: one lane of the byte-exact kernel
    t.data = a.data + nfull * a.bpc;
    t.len = tail;
    t.chunk_base = a.chunk_base + nfull;
    t.overlap_previous = false;
    if (verify) t.crc_be = a.crc_be + 4 * nfull;
    else t.out_be = a.out_be + 4 * nfull;
    return verify ? launch_t<0, true>(t, d_tables, 1, stream) : launch_t<0, false>(t, d_tables, 1, stream);
}

}  // namespace

// A packet stream whose chunks are R = bpc / 4096 whole rounds (64 KiB datanode packets at bpc 8192
// ... 65536; round 4). The pitch walk computes every 4096-byte piece's CRC densely into the piece
// scratch (packet p's pieces at 4 (p * upp + i)), the combine folds each chunk's R pieces and
// compares with (verify) or writes (compute) the word in the packet's own CRC region, key
// (packet << 32) | chunk; the last packet's short chunk, if any, takes the byte-exact kernel.
// Until round 4 these streams took the chunk-per-lane packet kernel.
hipError_t launch_stream_pieces(const ChunkLaunch &a, bool verify, const uint32_t *d_tables, const uint32_t *d_fold,
                                int grid_cap, hipStream_t stream, PieceScratch *ps) {
    const uint32_t R = a.bpc / kRoundBytes;
    const uint64_t upp = a.geom.upp;
    const uint64_t cpp = a.geom.pk_len / a.bpc;              // chunks per packet
    const uint64_t lfull = a.last_len / a.bpc;               // whole chunks of the last packet
    const uint64_t nfull = (a.npk - 1) * cpp + lfull;
    const uint64_t npieces = (a.npk - 1) * upp + (uint64_t(a.last_len) + kRoundBytes - 1) / kRoundBytes;
    const uint64_t cpitch = a.crc_pitch ? a.crc_pitch : a.pitch;
    unsigned b = 0;
    if (hipError_t e = piece_buffer(ps, npieces * 4, stream, &b); e != hipSuccess) return e;
    ChunkLaunch p = a;  // the pieces: a compute at bpc 4096 over the stream, words dense in the scratch
    p.bpc = kRoundBytes;
    p.out_be = ps->d[b];
    p.crc_be = ps->d[b];
    p.crc_pitch = upp * 4;
    p.check_short_tail = 1;
    hipError_t e = launch_stream_kernel(p, false, d_tables, d_fold, grid_cap, stream);
    if (e != hipSuccess) return e;
    if (nfull) {
        const uint64_t blocks = (nfull + 255) / 256;
        const int grid = int(blocks < 1024 ? blocks : 1024);
        if (verify)
            hipLaunchKernelGGL(crc32c_combine_pieces_kernel<true>, dim3(grid), dim3(256), 0, stream, ps->d[b], nfull,
                               R, d_fold, a.crc_be, nullptr, 0, a.result, cpp, cpitch);
        else
            hipLaunchKernelGGL(crc32c_combine_pieces_kernel<false>, dim3(grid), dim3(256), 0, stream, ps->d[b], nfull,
                               R, d_fold, nullptr, a.out_be, 0, a.result, cpp, cpitch);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    e = hipEventRecord(ps->used[b], stream);
    if (e != hipSuccess) return e;
    const uint64_t tail = a.last_len % a.bpc;
    if (tail == 0) return hipSuccess;
    const uint64_t lp = a.npk - 1;
    ChunkLaunch t{};  // the last packet's short chunk: one lane of the byte-exact kernel
    t.data = a.data + lp * a.pitch + lfull * a.bpc;
    t.len = tail;
    t.bpc = a.bpc;
    t.chunk_base = (lp << 32) | lfull;
    t.check_short_tail = a.check_short_tail;
    t.result = a.result;
    if (verify) t.crc_be = a.crc_be + lp * cpitch + 4 * lfull;
    else t.out_be = a.out_be + lp * cpitch + 4 * lfull;
    return verify ? launch_t<0, true>(t, d_tables, 1, stream) : launch_t<0, false>(t, d_tables, 1, stream);
}

hipError_t launch_chunks(const ChunkLaunch &a, bool verify, const uint32_t *d_tables,
                         const uint32_t *d_fold, int grid_cap, hipStream_t stream, PieceScratch *pieces) {
    const uint64_t chunks = (a.len + a.bpc - 1) / a.bpc;
    if (chunks == 0) return hipSuccess;
    const bool aligned = (reinterpret_cast<uintptr_t>(a.data) & 15u) == 0 &&
                         (reinterpret_cast<uintptr_t>(verify ? a.crc_be : a.out_be) & 3u) == 0;
    const uint64_t unit = a.bpc <= uint32_t(kRoundBytes) ? uint64_t(kRoundBytes) : a.bpc;
#if HDFS3_LAB
    if (g_variant == 123) pieces = nullptr;  // A/B: the multi-round kernel (before r3zf)
#endif
    // pieces + combine from 256 MiB per launch: 1 GiB at bpc 8192 / 16384 / 65536 172.7 / 173.5 / 174.4 us
    // against 196.0 / 200.6 / 209.1 for the multi-round kernel, but the combine's own launch (~6 us,
    // latency-bound) loses 0.9 us at 128 MiB (profiles/r03/reentry/r3zf_*.jsonl); chunk sizes the
    // multi-round kernel does not cover (12 KiB, 32 KiB, ...) take the pieces at every length
    const bool multi_round = a.bpc == 8192 || a.bpc == 16384 || a.bpc == 65536;
    if (pieces && aligned && a.bpc > uint32_t(kRoundBytes) && a.bpc % kRoundBytes == 0 && a.len >= a.bpc &&
        (!multi_round || a.len >= kPiecesMinBytes))
        return launch_pieces(a, verify, d_tables, d_fold, grid_cap, stream, pieces);
    if (aligned && a.len >= unit) {
        switch (a.bpc) {
        case 512: return launch_rv<512>(a, verify, d_tables, d_fold, grid_cap, stream);
        case 1024: return launch_rv<1024>(a, verify, d_tables, d_fold, grid_cap, stream);
        case 2048: return launch_rv<2048>(a, verify, d_tables, d_fold, grid_cap, stream);
        case 4096: return launch_rv<4096>(a, verify, d_tables, d_fold, grid_cap, stream);
        case 8192: return launch_rv<8192>(a, verify, d_tables, d_fold, grid_cap, stream);
        case 16384: return launch_rv<16384>(a, verify, d_tables, d_fold, grid_cap, stream);
        case 65536: return launch_rv<65536>(a, verify, d_tables, d_fold, grid_cap, stream);
        default: break;
        }
    }
    const uint64_t need = (chunks + kBlockThreads - 1) / kBlockThreads;
    const int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
    return verify ? launch_t<0, true>(a, d_tables, grid, stream)
                  : launch_t<0, false>(a, d_tables, grid, stream);
}

hipError_t launch_packets(const uint8_t *d_arena, const DevPacket *d_pk, uint64_t n, uint32_t bpc,
                          bool verify, int check_short_tail, unsigned long long *result,
                          const uint32_t *d_tables, int grid_cap, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    constexpr uint64_t kWaves = kBlockThreads / 64;
    const uint64_t need = (n + kWaves - 1) / kWaves;
    const int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
    if (verify)
        hipLaunchKernelGGL((crc32c_packets_kernel<true>), dim3(grid), dim3(kBlockThreads), 0,
                           stream, d_arena, nullptr, d_pk, n, bpc, check_short_tail, result,
                           d_tables);
    else
        hipLaunchKernelGGL((crc32c_packets_kernel<false>), dim3(grid), dim3(kBlockThreads), 0,
                           stream, d_arena, const_cast<uint8_t *>(d_arena), d_pk, n, bpc, 0,
                           result, d_tables);
    return hipGetLastError();
}

uint64_t plan_segments(DevSegment *h_seg, size_t n, uint32_t bpc, uint64_t *uniform) {
    uint64_t units = 0, u0 = n ? seg_units(h_seg[0].len, bpc) : 0;
    bool same = true;
    for (size_t i = 0; i < n; ++i) {
        h_seg[i].unit_begin = units;
        const uint64_t u = seg_units(h_seg[i].len, bpc);
        if (i + 1 < n && u != u0) same = false;
        units += u;
    }
    *uniform = same && u0 > 0 ? u0 : 0;
    return units;
}

bool segments_fast(const DevSegment *h_seg, size_t n, uint32_t bpc) {
    if (bpc != 512 && bpc != 1024 && bpc != 2048 && bpc != 4096) return false;
    for (size_t i = 0; i < n; ++i)
        if ((reinterpret_cast<uintptr_t>(h_seg[i].data) & 15u) || (reinterpret_cast<uintptr_t>(h_seg[i].crc) & 3u))
            return false;
    return true;
}

template <int BPC>
hipError_t launch_seg_t(const SegLaunch &L, bool verify, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                        hipStream_t s) {
#if HDFS3_LAB
    if (g_variant == 115)
        return verify ? launch_segments3<BPC, true, kLabPrio>(L, tab, fold, grid_cap, s)
                      : launch_segments3<BPC, false, kLabPrio>(L, tab, fold, grid_cap, s);
    if (g_variant == 117)
        return verify ? launch_segments3<BPC, true, kLabNoPrio>(L, tab, fold, grid_cap, s)
                      : launch_segments3<BPC, false, kLabNoPrio>(L, tab, fold, grid_cap, s);
    // 1024-thread workgroups at every size (production before round 6)
    if (g_variant == 161)
        return verify ? launch_segments3<BPC, true, 0, 1024>(L, tab, fold, grid_cap, s)
                      : launch_segments3<BPC, false, 0, 1024>(L, tab, fold, grid_cap, s);
#endif
    return verify ? launch_segments3<BPC, true>(L, tab, fold, grid_cap, s)
                  : launch_segments3<BPC, false>(L, tab, fold, grid_cap, s);
}

hipError_t launch_segments(const DevSegment *d_seg, uint32_t nseg, uint64_t units, uint64_t uniform,
                           uint32_t bpc, bool verify, int check_short_tail, unsigned long long *result,
                           const uint32_t *d_tables, const uint32_t *d_fold, int grid_cap, hipStream_t stream,
                           const DevSegment *h_inline, uint64_t stride, uint8_t *dense_words,
                           const uint32_t *unit_seg) {
    if (nseg == 0) return hipSuccess;
    SegLaunch L{};
    L.dense_words = dense_words;
    L.unit_seg = unit_seg;
    L.seg = d_seg;
    L.nseg = nseg;
    L.units = units;
    L.uniform = uniform;
    L.result = result;
    L.check_short_tail = check_short_tail;
    if (stride) {  // h_inline = {first packet, last packet}; the rest follow by pitch
        if (!h_inline || !uniform) return hipErrorInvalidValue;
        L.seg = nullptr;
        L.stride = stride;
        L.inl[0] = h_inline[0];
        L.inl[1] = h_inline[1];
    } else if (h_inline) {
        if (nseg > kInlineSegments) return hipErrorInvalidValue;
        L.seg = nullptr;
        for (uint32_t i = 0; i < nseg; ++i) L.inl[i] = h_inline[i];
    }
    switch (bpc) {
    case 512: return launch_seg_t<512>(L, verify, d_tables, d_fold, grid_cap, stream);
    case 1024: return launch_seg_t<1024>(L, verify, d_tables, d_fold, grid_cap, stream);
    case 2048: return launch_seg_t<2048>(L, verify, d_tables, d_fold, grid_cap, stream);
    case 4096: return launch_seg_t<4096>(L, verify, d_tables, d_fold, grid_cap, stream);
    default: return hipErrorInvalidValue;
    }
}

namespace {

// Descriptor lists at bpc = R x 4096 that are not one constant-pitch stream (round 6): the segmented
// kernel computes every 4096-byte piece of every segment densely (segment i's pieces from piece
// unit_begin_i, SegLaunch::dense_words), then this combine folds each chunk from its R pieces
// (crc32c_combine_pieces_kernel's fold) and compares with / writes the segment's own word c, key
// key_base + c. One wave per segment at a time (grid-stride), its lanes over the segment's chunks: a
// datanode packet holds few chunks at these sizes (5 of 12 KiB, 1 of 64 KiB).
template <bool VERIFY>
__global__ __launch_bounds__(256) void crc32c_combine_segment_pieces_kernel(const DevSegment *__restrict__ seg,
                                                                            uint32_t n,
                                                                            const uint8_t *__restrict__ piece_be,
                                                                            uint32_t bpc,
                                                                            const uint32_t *__restrict__ g_fold,
                                                                            unsigned long long *result) {
    uint32_t col[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) col[i] = g_fold[kFoldAdvance4096 + i];
    const uint32_t K = gf2_apply4(col, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    const uint32_t R = bpc / kRoundBytes;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = uint64_t(gridDim.x) * 4;
    for (uint64_t si = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); si < n; si += nwaves) {
        const DevSegment sd = seg[si];
        const uint64_t nfull = sd.len / bpc;
        for (uint64_t c = lane; c < nfull; c += 64) {
            const uint32_t *y = reinterpret_cast<const uint32_t *>(piece_be) + sd.unit_begin + c * R;
            uint32_t st = 0xFFFFFFFFu;
            for (uint32_t i = 0; i < R; ++i) st = gf2_apply4(col, st) ^ __builtin_bswap32(y[i]) ^ K;
            const uint32_t v = ~st;
            if constexpr (VERIFY) {
                if (__builtin_bswap32(*reinterpret_cast<const uint32_t *>(sd.crc + 4 * c)) != v)
                    atomicMax(result, ~(unsigned long long)(sd.key_base + c));
            } else {
                *reinterpret_cast<uint32_t *>(sd.crc + 4 * c) = __builtin_bswap32(v);
            }
        }
    }
}

// unit -> segment map of a long descriptor list (SegLaunch::unit_seg): one wave per segment at a time,
// its lanes over the segment's units (seg_units at ubpc: its whole chunks in 4 KiB units). A segmented
// kernel's wave steps nwaves units per round, past dozens of short segments, so without the map every
// round began with a binary search, a chain of ~15 dependent scalar loads (25k segments): 1 GiB of
// 12 KiB-chunk packets 327.3 -> 253.2 us verify, the pieces kernel 252 -> 166 us (profiles/r06/r6x_*,
// r6za_*). A 16-ary search (15 scalar loads per level) measured slower (430 us): the compiler issued
// them two at a time
__global__ __launch_bounds__(256) void crc32c_unit_map_kernel(const DevSegment *__restrict__ seg, uint32_t n,
                                                              uint32_t ubpc, uint32_t *__restrict__ map) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = uint64_t(gridDim.x) * 4;
    for (uint64_t si = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); si < n; si += nwaves) {
        const uint64_t ub = seg[si].unit_begin, len = seg[si].len;
        const uint64_t nu = (len / ubpc * ubpc + kRoundBytes - 1) / kRoundBytes;
        for (uint64_t t = lane; t < nu; t += 64) map[ub + t] = uint32_t(si);
    }
}

// Lists longer than this take the unit map (below it the search is a few loads and the map's launch
// is not worth it)
constexpr size_t kUnitMapMinSegments = 256;

// the descriptors' H2D copy: in-stream, or for long lists on the side stream so it runs under the previous
// launch (1 GiB of 32-64 KiB packets: 872 KB of descriptors)
hipError_t copy_descs(void *d, const void *h, size_t bytes, hipStream_t stream, const DescCopy *dc) {
    if (dc && dc->side && dc->copied && bytes >= kSideCopyMinBytes) {
        hipError_t e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, dc->side);
        if (e == hipSuccess) e = hipEventRecord(dc->copied, dc->side);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, dc->copied, 0);
        return e;
    }
    return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream);
}

// the segments' short last chunks (len % bpc bytes), one thread each
template <bool VERIFY>
__global__ __launch_bounds__(kBlockThreads) void crc32c_segment_tails_kernel(const DevSegment *__restrict__ seg,
                                                                             uint32_t n, uint32_t bpc,
                                                                             int check_short_tail,
                                                                             unsigned long long *result,
                                                                             const uint32_t *__restrict__ g_tab) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
    fill_tables(lds, g_tab);
    lds_barrier();
    const Lut t(lds);
    for (uint64_t i = uint64_t(blockIdx.x) * kBlockThreads + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * kBlockThreads) {
        const DevSegment sd = seg[i];
        const uint32_t tail = uint32_t(sd.len % bpc);
        if (!tail) continue;
        const uint64_t c = sd.len / bpc;
        const uint32_t v = ~crc_run_any(t, 0xFFFFFFFFu, sd.data + c * bpc, tail);
        const bool al = (reinterpret_cast<uintptr_t>(sd.crc) & 3u) == 0;
        if constexpr (VERIFY) {
            if (check_short_tail && load_be32(sd.crc + 4 * c, al) != v)
                atomicMax(result, ~(unsigned long long)(sd.key_base + c));
        } else {
            store_be32(sd.crc + 4 * c, v, al);
        }
    }
}

// h_stage[0..n) planned at 4096-byte units (unit_begin = the segment's first piece); the descriptors go
// to d_stage (always: the combine and the tails read them), *staged is set
hipError_t launch_segment_pieces(DevSegment *h_stage, DevSegment *d_stage, size_t n, uint64_t pieces_total,
                                 uint32_t bpc, bool verify, int check_short_tail, unsigned long long *result,
                                 const uint32_t *d_tables, const uint32_t *d_fold, int grid_cap,
                                 hipStream_t stream, PieceScratch *ps, uint64_t max_chunks, bool any_tail,
                                 bool *staged, const DescCopy *dc) {
    unsigned b = 0;
    // the piece words, then (long lists) the unit -> segment map
    const bool map = n > kUnitMapMinSegments && pieces_total;
    if (hipError_t e = piece_buffer(ps, (pieces_total ? pieces_total : 1) * (map ? 8 : 4), stream, &b);
        e != hipSuccess)
        return e;
    hipError_t e = copy_descs(d_stage, h_stage, n * sizeof(DevSegment), stream, dc);
    if (e != hipSuccess) return e;
    if (staged) *staged = true;
    uint32_t *unit_seg = nullptr;
    if (map) {
        unit_seg = reinterpret_cast<uint32_t *>(ps->d[b] + pieces_total * 4);
        const uint64_t want = (n + 3) / 4;
        hipLaunchKernelGGL(crc32c_unit_map_kernel, dim3(int(want < 2048 ? want : 2048)), dim3(256), 0, stream,
                           d_stage, uint32_t(n), uint32_t(kRoundBytes), unit_seg);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (pieces_total) {
        e = launch_segments(d_stage, uint32_t(n), pieces_total, 0, kRoundBytes, false, 1, nullptr, d_tables, d_fold,
                            grid_cap, stream, nullptr, 0, ps->d[b], unit_seg);
        if (e != hipSuccess) return e;
    }
    if (max_chunks) {
        const uint64_t want = (n + 3) / 4;  // 4 waves per workgroup, a segment per wave
        const int grid = int(want < 2048 ? want : 2048);
        if (verify)
            hipLaunchKernelGGL(crc32c_combine_segment_pieces_kernel<true>, dim3(grid), dim3(256), 0, stream, d_stage,
                               uint32_t(n), ps->d[b], bpc, d_fold, result);
        else
            hipLaunchKernelGGL(crc32c_combine_segment_pieces_kernel<false>, dim3(grid), dim3(256), 0, stream,
                               d_stage, uint32_t(n), ps->d[b], bpc, d_fold, result);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    e = hipEventRecord(ps->used[b], stream);
    if (e != hipSuccess) return e;
    if (!any_tail) return hipSuccess;
    const uint64_t blocks = (n + kBlockThreads - 1) / kBlockThreads;
    const int grid = int(blocks < uint64_t(grid_cap) ? blocks : uint64_t(grid_cap));
    if (verify)
        hipLaunchKernelGGL(crc32c_segment_tails_kernel<true>, dim3(grid), dim3(kBlockThreads), 0, stream, d_stage,
                           uint32_t(n), bpc, check_short_tail, result, d_tables);
    else
        hipLaunchKernelGGL(crc32c_segment_tails_kernel<false>, dim3(grid), dim3(kBlockThreads), 0, stream, d_stage,
                           uint32_t(n), bpc, 0, result, d_tables);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_packet_batch(const uint8_t *d_arena, const DevPacket *h_pk, size_t n, uint32_t bpc, bool verify,
                               int check_short_tail, unsigned long long *result, DevSegment *h_stage,
                               DevSegment *d_stage, const uint32_t *d_tables, const uint32_t *d_fold, int grid_cap,
                               hipStream_t stream, uint64_t arena_len, size_t *bad_index, bool overlap_previous,
                               WordScratch *ws, PieceScratch *pieces, bool *staged, const DescCopy *dc) {
    if (staged) *staged = false;
    if (n == 0) return hipSuccess;
    // one pass: descriptors, the alignment test of segments_fast and the unit plan of
    // plan_segments (16K packets per GiB: the host loop is on the call's critical path)
    bool fast = g_variant != 17 && (bpc == 512 || bpc == 1024 || bpc == 2048 || bpc == 4096);
    // bpc = R * 4096: the pitch walk's pieces + combine when the batch is a constant-pitch stream
    bool aligned = g_variant != 17 && (fast || (pieces && bpc > kRoundBytes && bpc % kRoundBytes == 0));
    const uint32_t ubpc = bpc <= uint32_t(kRoundBytes) ? bpc : uint32_t(kRoundBytes);
    uint64_t units = 0, u0 = seg_units(h_pk[0].data_len, ubpc);
    bool same = true;
    // constant pitch: packet i at data_off[0] + i*S, crc_off[0] + i*S, one data length
    // (the last may be shorter) -> the kernel derives every descriptor (SegLaunch::stride)
    const uint64_t pitch = n > 1 ? h_pk[1].data_off - h_pk[0].data_off : 0;
    bool strided = n > 1 && g_variant != 52 && pitch > 0 && pitch == h_pk[1].crc_off - h_pk[0].crc_off;
    // the same with the words at a pitch of their own (round 5: the output stream's batches, whose
    // words are dense at 4 x chunks per packet while the data sits in packet slots): the pitch walk
    // with ChunkLaunch::crc_pitch, so writer packets of whole rounds (bpc 1024 ... 65536: 64 KiB of
    // data) take the round kernel, and at bpc = R x 4096 its pieces + combine, instead of the
    // descriptor-array segmented kernel or (above 4 KiB) the chunk-per-lane packet kernel
    const uint64_t cpitch = n > 1 ? h_pk[1].crc_off - h_pk[0].crc_off : 0;
    bool dstrided = n > 1 && g_variant != 52 && pitch > 0 && h_pk[1].crc_off > h_pk[0].crc_off && (cpitch & 3) == 0;
    for (size_t i = 0; i < n; ++i) {
        if (bad_index) {  // bounds, fused into this pass (the API's only pass over pk[])
            const hdfs3crc::DevPacket &d = h_pk[i];
            const uint64_t chunks = (uint64_t(d.data_len) + bpc - 1) / bpc;
            if (d.data_off > arena_len || d.data_len > arena_len - d.data_off || d.crc_off > arena_len ||
                4 * chunks > arena_len - d.crc_off) {
                if (bad_index) *bad_index = i;
                return hipErrorInvalidValue;
            }
        }
        const uint8_t *data = d_arena + h_pk[i].data_off;
        const uint8_t *crc = d_arena + h_pk[i].crc_off;
        const uint64_t u = seg_units(h_pk[i].data_len, ubpc);
        const bool al = ((reinterpret_cast<uintptr_t>(data) & 15u) | (reinterpret_cast<uintptr_t>(crc) & 3u)) == 0;
        fast = fast && al;
        aligned = aligned && al;
        if (i + 1 < n && u != u0) same = false;
        strided = strided && h_pk[i].data_off == h_pk[0].data_off + i * pitch &&
                  h_pk[i].crc_off == h_pk[0].crc_off + i * pitch &&
                  (i + 1 == n || h_pk[i].data_len == h_pk[0].data_len);
        dstrided = dstrided && h_pk[i].data_off == h_pk[0].data_off + i * pitch &&
                   h_pk[i].crc_off == h_pk[0].crc_off + i * cpitch &&
                   (i + 1 == n || h_pk[i].data_len == h_pk[0].data_len);
        units += u;
    }
    PacketGeom geom;
    if (aligned && (strided || dstrided) && n > 1 &&
        packet_stream_ok(h_pk[0].data_len, h_pk[n - 1].data_len, n, bpc, d_arena + h_pk[0].data_off,
                         d_arena + h_pk[0].crc_off, pitch, &geom)) {
        ChunkLaunch a{};
        a.data = d_arena + h_pk[0].data_off;
        a.crc_be = d_arena + h_pk[0].crc_off;
        a.out_be = const_cast<uint8_t *>(d_arena) + h_pk[0].crc_off;
        a.bpc = bpc;
        a.result = result;
        a.check_short_tail = check_short_tail;
        a.pitch = pitch;
        a.crc_pitch = strided ? 0 : cpitch;
        a.npk = n;
        a.geom = geom;
        a.last_len = h_pk[n - 1].data_len;
        a.overlap_previous = overlap_previous && verify;
        const hipError_t e = launch_packet_stream(a, verify, d_tables, d_fold, grid_cap, stream, ws, pieces);
        if (e != hipErrorNotSupported) return e;
    }
    if (fast && strided && same && u0 > 0 && n > kInlineSegments) {
        const DevSegment ends[2] = {
            DevSegment{d_arena + h_pk[0].data_off, const_cast<uint8_t *>(d_arena) + h_pk[0].crc_off,
                       h_pk[0].data_len, 0, 0},
            DevSegment{d_arena + h_pk[n - 1].data_off, const_cast<uint8_t *>(d_arena) + h_pk[n - 1].crc_off,
                       h_pk[n - 1].data_len, (n - 1) * u0, uint64_t(n - 1) << 32}};
        return launch_segments(nullptr, uint32_t(n), units, u0, bpc, verify, check_short_tail, result, d_tables,
                               d_fold, grid_cap, stream, ends, pitch);
    }
    units = 0;
    for (size_t i = 0; i < n; ++i) {
        h_stage[i] = DevSegment{d_arena + h_pk[i].data_off, const_cast<uint8_t *>(d_arena) + h_pk[i].crc_off,
                                h_pk[i].data_len, units, uint64_t(i) << 32};
        units += seg_units(h_pk[i].data_len, ubpc);
    }
    // bpc = R x 4096, aligned, not one constant-pitch stream: piece CRCs over the segment list + the combine
    // (round 6; the chunk-per-lane packet kernel before, ~1 TiB/s)
    if (!fast && aligned && pieces && bpc > kRoundBytes && bpc % kRoundBytes == 0 && n < (size_t(1) << 31)) {
        uint64_t pieces_total = 0, max_chunks = 0;
        bool any_tail = false;
        for (size_t i = 0; i < n; ++i) {
            h_stage[i].unit_begin = pieces_total;
            pieces_total += h_stage[i].len / kRoundBytes;
            const uint64_t nf = h_stage[i].len / bpc;
            max_chunks = nf > max_chunks ? nf : max_chunks;
            any_tail = any_tail || (h_stage[i].len % bpc) != 0;
        }
        return launch_segment_pieces(h_stage, d_stage, n, pieces_total, bpc, verify, check_short_tail, result,
                                     d_tables, d_fold, grid_cap, stream, pieces, max_chunks, any_tail, staged, dc);
    }
    if (fast) {
        const uint64_t uniform = same && u0 > 0 ? u0 : 0;
        if (n > kInlineSegments) {
            hipError_t e = copy_descs(d_stage, h_stage, n * sizeof(DevSegment), stream, dc);
            if (e != hipSuccess) return e;
            if (staged) *staged = true;
        }
        if (n <= kInlineSegments)  // no descriptor copy in front of the kernel
            return launch_segments(nullptr, uint32_t(n), units, uniform, bpc, verify, check_short_tail, result,
                                   d_tables, d_fold, grid_cap, stream, h_stage);
        if (!uniform && n > kUnitMapMinSegments && pieces && units) {
            // a long ragged list: the unit -> segment map in the piece scratch (4 B per 4 KiB unit)
            // instead of a binary search per round; 1 GiB of 32-64 KiB packets at bpc 512: 313.6 ->
            // 219.7 us verify (profiles/r06/r6za_partial_rate.jsonl, r6zb_partial_rate.jsonl)
            unsigned b = 0;
            if (hipError_t e = piece_buffer(pieces, units * 4, stream, &b); e != hipSuccess) return e;
            uint32_t *unit_seg = reinterpret_cast<uint32_t *>(pieces->d[b]);
            const uint64_t want = (n + 3) / 4;
            hipLaunchKernelGGL(crc32c_unit_map_kernel, dim3(int(want < 2048 ? want : 2048)), dim3(256), 0, stream,
                               d_stage, uint32_t(n), ubpc, unit_seg);
            hipError_t e = hipGetLastError();
            if (e == hipSuccess)
                e = launch_segments(d_stage, uint32_t(n), units, 0, bpc, verify, check_short_tail, result, d_tables,
                                    d_fold, grid_cap, stream, nullptr, 0, nullptr, unit_seg);
            if (e == hipSuccess) e = hipEventRecord(pieces->used[b], stream);
            return e;
        }
        return launch_segments(d_stage, uint32_t(n), units, uniform, bpc, verify, check_short_tail, result,
                               d_tables, d_fold, grid_cap, stream);
    }
    // variant 17 (A/B) or unaligned / other chunk sizes: one wave per packet
    DevPacket *hp = reinterpret_cast<DevPacket *>(h_stage);
    for (size_t i = 0; i < n; ++i) hp[i] = h_pk[i];
    hipError_t e = copy_descs(d_stage, hp, n * sizeof(DevPacket), stream, dc);
    if (e != hipSuccess) return e;
    if (staged) *staged = true;
    return launch_packets(d_arena, reinterpret_cast<const DevPacket *>(d_stage), n, bpc, verify, check_short_tail,
                          result, d_tables, grid_cap, stream);
}

}  // namespace hdfs3crc
