// gfx950 (CDNA4) CRC32C kernels for libhdfs3's per-chunk checksum path.
//
// Replaces the per-chunk reset/update/getValue loops of
//   RemoteBlockReader::verifyChecksum   (src/client/RemoteBlockReader.cpp:306-326)
//   LocalBlockReader::readAndVerify     (src/client/LocalBlockReader.cpp:138-163)
//   OutputStreamImpl::appendInternal    (src/client/OutputStreamImpl.cpp:298-359)
// with one launch over a whole batch of chunks.
//
// Mapping: one chunk per lane (chunks are independent, so no cross-lane fold is
// needed). Each lane walks its chunk in 16-byte loads and runs slice-by-4 table
// CRC: per 32-bit word, 4 LDS lookups. LDS is the co-bottleneck with HBM: a
// lookup per payload byte is 6-7e12 lookups/s at the HBM roofline, so the four
// 1 KiB slice tables are REPLICATED 32x across the LDS banks and lane l always
// reads copy l%32: every ds_read_b32 half-wave hits 32 distinct banks, i.e. it is
// conflict-free whatever the data. The image is 128 KiB, so one 1024-thread
// workgroup owns a CU.
//
// LDS image (byte address):  rowset*64K + entry*256 + half*128 + copy*4
//   slice 0 -> rowset 0 half 0,  slice 1 -> rowset 0 half 1,
//   slice 2 -> rowset 1 half 0,  slice 3 -> rowset 1 half 1.
// A 256-byte entry stride puts the table index in address byte 1, so ONE
// v_perm_b32 builds a lookup address from the CRC state and a per-lane base
// (bytes 0 and 2), and v_bitop3_b32 folds three lookups per instruction: a
// 32-bit word costs 4 v_perm + 2 v_bitop3 + 4 ds_read_b32.
#include "crc32c_kernels.h"
#include "crc32c_tables.h"

namespace hdfs3crc {
namespace {

constexpr int kCopies = 32;                                   // one per ds_read_b32 bank
constexpr int kLdsBytes = 128 * 1024;                         // 2 rowsets x 256 entries x 256 B
constexpr int kLdsSlots = kLdsBytes / 16;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Fill the replicated image from the 4 KiB global table image (slice-major,
// 256 words per slice). Consecutive lanes write consecutive 16-byte slots, so
// each ds_write_b128 lane group stores 128 contiguous bytes (conflict-free).
// Split in two so the caller can put its first data loads between the table
// fetch and the LDS stores (vmcnt is in-order: loads issued after the table
// words do not have to land before the stores).
constexpr int kFillPerThread = kLdsSlots / kBlockThreads;

__device__ __forceinline__ void fetch_tables(uint32_t (&v)[kFillPerThread],
                                             const uint32_t *__restrict__ g_tab) {
#pragma unroll
    for (int i = 0; i < kFillPerThread; ++i) {
        const int s = i * kBlockThreads + threadIdx.x;
        const int rowset = s >> 12, entry = (s >> 4) & 255, half = (s >> 3) & 1;
        v[i] = g_tab[(rowset * 2 + half) * kTableEntries + entry];
    }
}

__device__ __forceinline__ void store_tables(uint32_t *lds, const uint32_t (&v)[kFillPerThread]) {
    u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
#pragma unroll
    for (int i = 0; i < kFillPerThread; ++i) l4[i * kBlockThreads + threadIdx.x] = u32x4{v[i], v[i], v[i], v[i]};
}

__device__ __forceinline__ void fill_tables(uint32_t *lds, const uint32_t *__restrict__ g_tab) {
    uint32_t v[kFillPerThread];
    fetch_tables(v, g_tab);
    store_tables(lds, v);
}

// LDS writes visible to the whole workgroup. Written as asm so the compiler does
// not drain the data loads already in flight (a __syncthreads() would add vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct Lut {
    const uint8_t *lds;
    uint32_t base[4];  // per-slice lane base: rowset<<16 | half<<7 | lane*4

    __device__ __forceinline__ explicit Lut(const uint32_t *l) : lds(reinterpret_cast<const uint8_t *>(l)) {
        const uint32_t lane4 = (threadIdx.x & (kCopies - 1)) * 4;
        base[0] = lane4;
        base[1] = lane4 | 0x80u;
        base[2] = lane4 | 0x10000u;
        base[3] = lane4 | 0x10080u;
    }
    // T[slice][byte k of x]: address = {0, base.byte2, x.byte k, base.byte0}.
    template <int K>
    __device__ __forceinline__ uint32_t at(int slice, uint32_t x) const {
        const uint32_t addr = __builtin_amdgcn_perm(x, base[slice], 0x0C020000u | ((4u + K) << 8));
        return *reinterpret_cast<const uint32_t *>(lds + addr);
    }
    // x = state ^ word; returns the state after the word, pre-xored with `next`.
    __device__ __forceinline__ uint32_t word(uint32_t x, uint32_t next) const {
        return xor3(xor3(at<0>(3, x), at<1>(2, x), at<2>(1, x)), at<3>(0, x), next);
    }
    // One byte (SWCrc32c.cpp:102): crc = T0[(crc ^ b) & 0xFF] ^ (crc >> 8).
    __device__ __forceinline__ uint32_t byte(uint32_t c, uint32_t b) const {
        return at<0>(0, c ^ b) ^ (c >> 8);
    }
    // Plain-state helpers for the irregular paths.
    __device__ __forceinline__ uint32_t word_state(uint32_t c, uint32_t w) const { return word(c ^ w, 0); }
    __device__ __forceinline__ uint32_t vec_state(uint32_t c, u32x4 v) const {
        uint32_t x = c ^ v.x;
        x = word(x, v.y);
        x = word(x, v.z);
        x = word(x, v.w);
        return word(x, 0);
    }
};

__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}

// Arbitrary pointer/length run, alignment dispatched per call (packet arenas put
// data at odd offsets; the short tail chunk of a block). `n` bytes from `p`.
__device__ uint32_t crc_run_any(const Lut &t, uint32_t c, const uint8_t *p, uint32_t n) {
    // bytes up to 4-byte alignment
    while (n && (reinterpret_cast<uintptr_t>(p) & 3u)) {
        c = t.byte(c, *p++);
        --n;
    }
    if ((reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
        for (; n >= 16; n -= 16, p += 16) c = t.vec_state(c, ld16(p));
    }
    for (; n >= 4; n -= 4, p += 4) c = t.word_state(c, *reinterpret_cast<const uint32_t *>(p));
    for (; n; --n) c = t.byte(c, *p++);
    return c;
}

__device__ __forceinline__ uint32_t load_be32(const uint8_t *p, bool aligned4) {
    if (aligned4) return __builtin_bswap32(*reinterpret_cast<const uint32_t *>(p));
    return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}
__device__ __forceinline__ void store_be32(uint8_t *p, uint32_t v, bool aligned4) {
    if (aligned4) {
        *reinterpret_cast<uint32_t *>(p) = __builtin_bswap32(v);
        return;
    }
    p[0] = uint8_t(v >> 24); p[1] = uint8_t(v >> 16); p[2] = uint8_t(v >> 8); p[3] = uint8_t(v);
}

// Main chunk kernel. BPC > 0: compile-time bytes-per-checksum (512/1024/2048/4096)
// with 16-byte aligned data; BPC == 0: run-time bpc / any alignment.
//
// Each lane streams its chunk as 128-byte lines (8 x global_load_dwordx4): the
// loads of line l+1 (or of the next chunk's first line) are issued, and pinned
// in place by a sched_barrier, before line l is consumed, so every lane keeps
// 128-256 B in flight (256 KiB per CU) while it works through the tables.
template <int BPC, bool VERIFY>
__global__ __launch_bounds__(kBlockThreads) void crc32c_chunks_kernel(ChunkLaunch a,
                                                                      const uint32_t *__restrict__ g_tab) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
    const uint32_t bpc = BPC > 0 ? uint32_t(BPC) : a.bpc;
    const uint64_t nfull = a.len / bpc;
    const uint64_t stride = uint64_t(gridDim.x) * kBlockThreads;
    uint64_t chunk = uint64_t(blockIdx.x) * kBlockThreads + threadIdx.x;
    const bool crc_al4 = (reinterpret_cast<uintptr_t>(VERIFY ? a.crc_be : a.out_be) & 3u) == 0;

    u32x4 cur[8];
    uint32_t tv[kFillPerThread];
    fetch_tables(tv, g_tab);
    if constexpr (BPC > 0) {
        // First line in flight before the table fill so HBM latency overlaps it.
        // Unconditional (idle lanes re-read the last chunk; host ensures nfull >= 1)
        // so the waitcnt pass can count it precisely and not drain it at the fill.
        const uint64_t first = chunk < nfull ? chunk : nfull - 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) cur[i] = ld16(a.data + first * BPC + 16 * i);
        __builtin_amdgcn_sched_barrier(0);
    }
    store_tables(lds, tv);
    lds_barrier();
    const Lut t(lds);

    for (; chunk < nfull; chunk += stride) {
        const uint8_t *p = a.data + chunk * bpc;
        uint32_t c;
        // Stored word requested first: it is older than the prefetches below, so
        // waiting for it never drains the next chunk's loads (vmcnt is in-order).
        uint32_t want = 0;
        if constexpr (VERIFY) {
            if constexpr (BPC > 0)  // fast path: host guarantees a 4-byte aligned CRC array
                want = *reinterpret_cast<const uint32_t *>(a.crc_be + 4 * chunk);
            else
                want = load_be32(a.crc_be + 4 * chunk, crc_al4);
        }
        if constexpr (BPC > 0) {
            constexpr int kLines = BPC / 128;
            const uint64_t next_chunk = chunk + stride;
            // Last line prefetches the next chunk's first line; with no next chunk
            // it re-reads this chunk's (cache-resident) first line instead of
            // branching, so the load set stays unconditional and register-renamed.
            const uint8_t *pnext = next_chunk < nfull ? a.data + next_chunk * BPC : p;
            uint32_t x = 0xFFFFFFFFu ^ cur[0].x;
#pragma unroll
            for (int l = 0; l < kLines; ++l) {
                u32x4 nxt[8];
                const uint8_t *src = l + 1 < kLines ? p + 128 * (l + 1) : pnext;
#pragma unroll
                for (int i = 0; i < 8; ++i) nxt[i] = ld16(src + 16 * i);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    x = t.word(x, cur[i].y);
                    x = t.word(x, cur[i].z);
                    x = t.word(x, cur[i].w);
                    const uint32_t follow = i < 7 ? cur[i + 1 < 8 ? i + 1 : 7].x
                                                  : (l + 1 < kLines ? nxt[0].x : 0u);
                    x = t.word(x, follow);
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) cur[i] = nxt[i];
            }
            c = x;
        } else {
            c = crc_run_any(t, 0xFFFFFFFFu, p, bpc);
        }
        c = ~c;
        if constexpr (VERIFY) {
            if (BPC > 0) want = __builtin_bswap32(want);
            if (want != c)
                atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
        } else {
            store_be32(a.out_be + 4 * chunk, c, BPC > 0 || crc_al4);
        }
    }
    // The lane whose stride sequence lands exactly on nfull owns the short tail chunk.
    const uint32_t tail = uint32_t(a.len - nfull * bpc);
    if (tail && chunk == nfull) {
        const uint32_t c = ~crc_run_any(t, 0xFFFFFFFFu, a.data + nfull * bpc, tail);
        if constexpr (VERIFY) {
            if (a.check_short_tail && load_be32(a.crc_be + 4 * nfull, crc_al4) != c)
                atomicMax(a.result, ~(unsigned long long)(a.chunk_base + nfull));
        } else {
            store_be32(a.out_be + 4 * nfull, c, crc_al4);
        }
    }
}

// Packet kernel: one wave per packet (grid-stride over packets), lanes over that
// packet's chunks. Result key = (packet << 32 | chunk), atomicMax of its complement
// keeps the lexicographically first bad (packet, chunk).
template <bool VERIFY>
__global__ __launch_bounds__(kBlockThreads) void crc32c_packets_kernel(
    const uint8_t *arena_c, uint8_t *arena_w, const DevPacket *__restrict__ pk,
    uint64_t n, uint32_t bpc, int check_short_tail, unsigned long long *result,
    const uint32_t *__restrict__ g_tab) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
    fill_tables(lds, g_tab);
    lds_barrier();
    const Lut t(lds);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = uint64_t(gridDim.x) * (kBlockThreads / 64);
    for (uint64_t w = uint64_t(blockIdx.x) * (kBlockThreads / 64) + (threadIdx.x >> 6); w < n;
         w += waves) {
        const DevPacket d = pk[w];
        const uint32_t chunks = (d.data_len + bpc - 1) / bpc;
        const uint8_t *data = arena_c + d.data_off;
        const bool al4 = (reinterpret_cast<uintptr_t>(arena_c + d.crc_off) & 3u) == 0;
        for (uint32_t k = lane; k < chunks; k += 64) {
            const uint32_t off = k * bpc;
            const uint32_t sz = d.data_len - off < bpc ? d.data_len - off : bpc;
            const uint32_t c = ~crc_run_any(t, 0xFFFFFFFFu, data + off, sz);
            if constexpr (VERIFY) {
                if ((sz == bpc || check_short_tail) &&
                    load_be32(arena_c + d.crc_off + 4ull * k, al4) != c)
                    atomicMax(result, ~((uint64_t(w) << 32) | k));
            } else {
                store_be32(arena_w + d.crc_off + 4ull * k, c, al4);
            }
        }
    }
}

// ---- measurement-only kernels ------------------------------------------------

// Coalesced streaming read (1 KiB per wave-instruction): the achievable HBM read
// ceiling the CRC kernel is compared with.
__global__ __launch_bounds__(256) void stream_read_kernel(const uint8_t *__restrict__ d,
                                                          uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const u32x4 a = ld16(d + 16 * i), b = ld16(d + 16 * (i + stride));
        const u32x4 c = ld16(d + 16 * (i + 2 * stride)), e = ld16(d + 16 * (i + 3 * stride));
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ e.x ^ e.y ^
               e.z ^ e.w;
    }
    for (; i < n16; i += stride) {
        const u32x4 a = ld16(d + 16 * i);
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // keep the loads live
}

// The CRC kernel's exact access pattern (chunk per lane, 128 B lines, one-line
// prefetch) with the table arithmetic replaced by xor.
template <int BPC>
__global__ __launch_bounds__(kBlockThreads) void lane_read_kernel(const uint8_t *__restrict__ d,
                                                                  uint64_t nchunks, uint32_t *sink) {
    const uint64_t stride = uint64_t(gridDim.x) * kBlockThreads;
    uint32_t acc = 0;
    for (uint64_t chunk = uint64_t(blockIdx.x) * kBlockThreads + threadIdx.x; chunk < nchunks;
         chunk += stride) {
        const uint8_t *p = d + chunk * BPC;
#pragma unroll
        for (int l = 0; l < BPC / 128; ++l) {
            u32x4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = ld16(p + 128 * l + 16 * i);
#pragma unroll
            for (int i = 0; i < 8; ++i) acc = (acc ^ v[i].x ^ v[i].y ^ v[i].z ^ v[i].w) * 3u;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <int BPC, bool V>
hipError_t launch_t(const ChunkLaunch &a, const uint32_t *tab, int grid, hipStream_t s) {
    hipLaunchKernelGGL((crc32c_chunks_kernel<BPC, V>), dim3(grid), dim3(kBlockThreads), 0, s, a,
                       tab);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_chunks(const ChunkLaunch &a, bool verify, const uint32_t *d_tables,
                         int grid_cap, hipStream_t stream) {
    const uint64_t chunks = (a.len + a.bpc - 1) / a.bpc;
    if (chunks == 0) return hipSuccess;
    const uint64_t need = (chunks + kBlockThreads - 1) / kBlockThreads;
    const int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
    const bool al16 = (reinterpret_cast<uintptr_t>(a.data) & 15u) == 0 &&
                      (reinterpret_cast<uintptr_t>(verify ? a.crc_be : a.out_be) & 3u) == 0;
    if (al16 && a.len >= a.bpc) {
        switch (a.bpc) {
        case 512: return verify ? launch_t<512, true>(a, d_tables, grid, stream)
                                : launch_t<512, false>(a, d_tables, grid, stream);
        case 1024: return verify ? launch_t<1024, true>(a, d_tables, grid, stream)
                                 : launch_t<1024, false>(a, d_tables, grid, stream);
        case 2048: return verify ? launch_t<2048, true>(a, d_tables, grid, stream)
                                 : launch_t<2048, false>(a, d_tables, grid, stream);
        case 4096: return verify ? launch_t<4096, true>(a, d_tables, grid, stream)
                                 : launch_t<4096, false>(a, d_tables, grid, stream);
        default: break;
        }
    }
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

hipError_t launch_stream_read(const uint8_t *d, uint64_t len, uint32_t *sink, int grid,
                              hipStream_t stream) {
    hipLaunchKernelGGL(stream_read_kernel, dim3(grid), dim3(256), 0, stream, d, len / 16, sink);
    return hipGetLastError();
}

hipError_t launch_lane_read(const uint8_t *d, uint64_t len, uint32_t bpc, uint32_t *sink,
                            int grid_cap, hipStream_t stream) {
    const uint64_t chunks = len / bpc;
    const uint64_t need = (chunks + kBlockThreads - 1) / kBlockThreads;
    const int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
    switch (bpc) {
    case 512:
        hipLaunchKernelGGL(lane_read_kernel<512>, dim3(grid), dim3(kBlockThreads), 0, stream, d,
                           chunks, sink);
        break;
    case 2048:
        hipLaunchKernelGGL(lane_read_kernel<2048>, dim3(grid), dim3(kBlockThreads), 0, stream, d,
                           chunks, sink);
        break;
    case 4096:
        hipLaunchKernelGGL(lane_read_kernel<4096>, dim3(grid), dim3(kBlockThreads), 0, stream, d,
                           chunks, sink);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace hdfs3crc
