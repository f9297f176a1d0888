// Device code of the gfx950 CRC32C kernels and their launch templates, shared by the
// production translation unit (crc32c_kernels.hip) and the A/B experiments
// (crc32c_experiments.hip). Internal; not installed.
#pragma once
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
#include <hip/hip_ext.h>

#include <type_traits>

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

// Default cache policy: measured 2.4x faster than nontemporal (`nt`) loads for the
// chunk-per-lane pattern and no slower for coalesced rounds (tools/sweep.py).
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    return *reinterpret_cast<const u32x4 *>(p);
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

// crc_run_any for a 16-byte aligned run: 128-byte lines whose 8 loads are issued
// together, then the remaining 16-byte pieces (again issued together), then words and
// bytes. One load latency per line instead of one per 16 bytes: the segmented kernel's
// slow pass runs it on one lane per chunk while the rest of the wave waits.
__device__ uint32_t crc_run_lines(const Lut &t, uint32_t c, const uint8_t *p, uint32_t n) {
    for (; n >= 128; n -= 128, p += 128) {
        u32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = ld16(p + 16 * i);
#pragma unroll
        for (int i = 0; i < 8; ++i) c = t.vec_state(c, v[i]);
    }
    const uint32_t k = n / 16;
    u32x4 v[7];
#pragma unroll
    for (int i = 0; i < 7; ++i)
        if (uint32_t(i) < k) v[i] = ld16(p + 16 * i);
#pragma unroll
    for (int i = 0; i < 7; ++i)
        if (uint32_t(i) < k) c = t.vec_state(c, v[i]);
    p += 16 * k;
    n -= 16 * k;
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

// ---- round kernel (the fast path) -------------------------------------------
//
// Work is cut into ROUNDS of 4 KiB of contiguous data, one round per wave at a
// time. A round is fetched with 4 perfectly coalesced global_load_dwordx4 (1 KiB
// each) and then regrouped in registers so that lane l owns the 64 contiguous bytes
// [64l, 64l+64) of the round:
//   instruction t gives lane (row r = l/16, c = l%16) the 16-byte piece 64t+4c+r;
//   lane (row s, c) needs pieces 64s+4c+q in register q  =>  a 4x4 transpose between
//   the wave's four 16-lane rows and the four load registers, done by one
//   v_permlane32_swap stage (rows {0,1} <-> {2,3}) and one v_permlane16_swap stage
//   (odd <-> even rows): 16 swaps per round, no LDS traffic.
// Each lane then runs slice-by-4 over its 16 words. A chunk of bpc <= 4096 bytes is
// G = bpc/64 consecutive lanes; lane j of a chunk advances its partial state over
// the (G-1-j)*64 bytes that follow its segment with a lane-specific 32x32 GF(2)
// matrix held in VGPRs (crc(A||B) = shift_|B|(crc(A)) ^ crc0(B)), the G states are
// xor-reduced with DPP / permlane swaps, and lane j == 0 finishes the chunk.
// For bpc a multiple of 4096 a wave walks the chunk's rounds in order and folds
// round results with the uniform 4096-byte advance.

constexpr int kRoundBytes = 4096;
constexpr int kWavesPerBlock = kBlockThreads / 64;

struct Round {
    uint32_t w[4][4];  // [load register][dword]
};

template <bool NT = false>
__device__ __forceinline__ void load_round(Round &r, const uint8_t *base, uint32_t lane_off) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const u32x4 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base + 1024 * t + lane_off))
                           : ld16(base + 1024 * t + lane_off);
        r.w[t][0] = v.x;
        r.w[t][1] = v.y;
        r.w[t][2] = v.z;
        r.w[t][3] = v.w;
    }
}

// A wave-uniform 64-bit value made provably uniform (two v_readfirstlane): downstream
// arithmetic then stays in SGPRs/SALU instead of 64-bit VALU per use.
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(x));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(x >> 32));
    return (uint64_t(hi) << 32) | lo;
}

// Same, through a buffer resource built from the wave-uniform round base (scalar
// registers, made provably uniform by readfirstlane: cdna_hip_programming.md T8/T20).
// The lane's constant byte offset is the only VGPR operand, so no 64-bit VGPR address
// temporaries exist that the allocator could alias with in-flight load destinations
// (which made the compiler drain the previous round's loads before each prefetch).
template <bool NT>
__device__ __forceinline__ void load_round_buf(Round &r, const uint8_t *base, uint32_t lane_off) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(b));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(b >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>((uint64_t(hi) << 32) | lo), 0, 4096, 0x00020000);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + 1024 * t, 0, NT ? 2 : 0);
        r.w[t][0] = v.x;
        r.w[t][1] = v.y;
        r.w[t][2] = v.z;
        r.w[t][3] = v.w;
    }
}

template <bool NT, bool BUF>
__device__ __forceinline__ void load_any(Round &r, const uint8_t *base, uint32_t lane_off) {
    if constexpr (BUF) load_round_buf<NT>(r, base, lane_off);
    else load_round<NT>(r, base, lane_off);
}

__device__ __forceinline__ void swap32(uint32_t &a, uint32_t &b) {
    const auto p = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = p[0];
    b = p[1];
}
__device__ __forceinline__ void swap16(uint32_t &a, uint32_t &b) {
    const auto p = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = p[0];
    b = p[1];
}

// (row, register) 4x4 transpose, see above.
__device__ __forceinline__ void regroup(Round &r) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        swap32(r.w[0][k], r.w[2][k]);
        swap32(r.w[1][k], r.w[3][k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        swap16(r.w[0][k], r.w[1][k]);
        swap16(r.w[2][k], r.w[3][k]);
    }
}

// y = M x over GF(2), M given by its 32 columns.
__device__ __forceinline__ uint32_t gf2_apply(const uint32_t (&col)[32], uint32_t x) {
    uint32_t y = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t m = uint32_t(int32_t(x << (31 - i)) >> 31);
        y ^= m & col[i];
    }
    return y;
}

// Same product, 4 independent accumulators and one v_bitop3 (y ^ (m & col), truth
// table 0x78 over {S0,S1,S2}) per bit: 64 VALU in chains of 8 instead of 96 in one chain.
__device__ __forceinline__ uint32_t gf2_apply4(const uint32_t (&col)[32], uint32_t x) {
    uint32_t y[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t m = uint32_t(int32_t(x << (31 - i)) >> 31);
        y[i & 3] = __builtin_amdgcn_bitop3_b32(y[i & 3], m, col[i], 0x78);
    }
    return xor3(y[0], y[1], y[2]) ^ y[3];
}

template <int DPP>
__device__ __forceinline__ uint32_t dpp_xor(uint32_t v) {
    // bound_ctrl: every lane of these patterns has a source; it lets the DPP combiner fold the
    // move into the xor (v_xor_b32_dpp), row_half_mirror included
    return v ^ uint32_t(__builtin_amdgcn_update_dpp(0, int(v), DPP, 0xF, 0xF, true));
}

// XOR-reduce over aligned groups of G lanes; the group total lands in (at least) the
// group's first lane.
template <int G>
__device__ __forceinline__ uint32_t group_xor(uint32_t v) {
    v = dpp_xor<0xB1>(v);   // quad_perm [1,0,3,2]
    v = dpp_xor<0x4E>(v);   // quad_perm [2,3,0,1]
    v = dpp_xor<0x141>(v);  // row_half_mirror: 8-lane total
    if constexpr (G >= 16) v = dpp_xor<0x140>(v);  // row_mirror: 16-lane total
    if constexpr (G >= 32) {
        uint32_t a = v, b = v;
        swap16(a, b);  // b's even rows now hold the odd rows' totals
        v ^= b;
    }
    if constexpr (G >= 64) {
        uint32_t a = v, b = v;
        swap32(a, b);  // b's lower half now holds the upper half's total
        v ^= b;
    }
    return v;
}

template <int BPC, bool VERIFY, int DEPTH, bool FOLD4>
__global__ __launch_bounds__(kBlockThreads) void crc32c_rounds_kernel(ChunkLaunch a,
                                                                      const uint32_t *__restrict__ g_tab,
                                                                      const uint32_t *__restrict__ g_fold) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
    constexpr int kUnit = BPC <= kRoundBytes ? kRoundBytes : BPC;  // bytes per wave work unit
    constexpr int kRoundsPerUnit = kUnit / kRoundBytes;
    constexpr int G = BPC <= kRoundBytes ? BPC / 64 : 64;           // lanes per chunk in a round
    constexpr int kChunksPerUnit = BPC <= kRoundBytes ? kRoundBytes / BPC : 1;
    constexpr int kFoldSet = G == 8 ? 0 : G == 16 ? 1 : G == 32 ? 2 : 3;
    constexpr int kFoldOff[4] = {0, 8, 24, 56};

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane % G;
    const uint32_t lane_off = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint64_t nunits = a.len / kUnit;
    const uint64_t nwaves = uint64_t(gridDim.x) * kWavesPerBlock;
    const uint64_t wave = uint64_t(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
    // this wave's rounds: k = 0..K-1 -> unit wave + (k / RPU) * nwaves, sub-round k % RPU
    const uint64_t my_units = wave < nunits ? (nunits - wave + nwaves - 1) / nwaves : 0;
    const uint64_t K = my_units * kRoundsPerUnit;
    const bool crc_al4 = (reinterpret_cast<uintptr_t>(VERIFY ? a.crc_be : a.out_be) & 3u) == 0;
    // byte offset of round k; rounds past the end re-read the wave's last round
    // (cache-resident) so every prefetch stays unconditional
    auto round_ptr = [&](uint64_t k) -> const uint8_t * {
        if (K == 0) return a.data;  // host guarantees nunits >= 1; idle wave reads unit 0
        const uint64_t kk = k < K ? k : K - 1;
        return a.data + (wave + (kk / kRoundsPerUnit) * nwaves) * kUnit + (kk % kRoundsPerUnit) * kRoundBytes;
    };

    // small cache-resident reads first (tables, fold columns), then the first two
    // rounds: the in-order vmcnt then lets the table fill proceed while rounds land
    uint32_t col[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) col[i] = g_fold[(kFoldOff[kFoldSet] + j) * 32 + i];
    uint32_t tv[kFillPerThread];
    fetch_tables(tv, g_tab);
    __builtin_amdgcn_sched_barrier(0);
    Round b0, b1, b2;
    load_round(b0, round_ptr(0), lane_off);
    if constexpr (DEPTH == 2) load_round(b1, round_ptr(1), lane_off);
    __builtin_amdgcn_sched_barrier(0);
    store_tables(lds, tv);
    lds_barrier();
    const Lut t(lds);

    uint32_t acc = 0;
    // One round: issue the stored CRC word and the prefetch of round k+DEPTH into
    // `pf`, then consume `cur`.
    auto step = [&](Round &cur, Round &pf, uint64_t k) {
        const uint32_t r = uint32_t(k % kRoundsPerUnit);
        const uint64_t unit = wave + (k / kRoundsPerUnit) * nwaves;
        const uint64_t chunk = unit * kChunksPerUnit + lane / G;
        uint32_t want = 0;
        if constexpr (VERIFY) {
            // every lane of a chunk reads its word (one broadcast access), issued before
            // the prefetch so that waiting for it never drains the prefetch (vmcnt is in-order)
            want = *reinterpret_cast<const uint32_t *>(a.crc_be + 4 * chunk);
        }
        load_round(pf, round_ptr(k + DEPTH), lane_off);
        __builtin_amdgcn_sched_barrier(0);
        regroup(cur);
        uint32_t x = ((j == 0 && r == 0) ? 0xFFFFFFFFu : 0u) ^ cur.w[0][0];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            x = t.word(x, cur.w[q][1]);
            x = t.word(x, cur.w[q][2]);
            x = t.word(x, cur.w[q][3]);
            x = t.word(x, q < 3 ? cur.w[q < 3 ? q + 1 : 3][0] : 0u);
        }
        uint32_t y = group_xor<G>(FOLD4 ? gf2_apply4(col, x) : gf2_apply(col, x));
        if constexpr (kRoundsPerUnit > 1) {
            if (r > 0) {
                uint32_t k4096[32];
#pragma unroll
                for (int i = 0; i < 32; ++i) k4096[i] = g_fold[kFoldAdvance4096 + i];
                y ^= gf2_apply(k4096, acc);
            }
        }
        acc = y;
        if (r == kRoundsPerUnit - 1 && j == 0) {
            const uint32_t c = ~acc;
            if constexpr (VERIFY) {
                if (__builtin_bswap32(want) != c)
                    atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
            } else {
                *reinterpret_cast<uint32_t *>(a.out_be + 4 * chunk) = __builtin_bswap32(c);
            }
        }
    };
    // (DEPTH+1)-buffer ring unrolled so the buffers rotate by renaming (a loop-carried
    // register copy would make the compiler wait for the youngest prefetch)
    if constexpr (DEPTH == 2) {
        for (uint64_t k = 0; k < K; k += 3) {
            step(b0, b2, k);
            if (k + 1 >= K) break;
            step(b1, b0, k + 1);
            if (k + 2 >= K) break;
            step(b2, b1, k + 2);
        }
    } else {
        for (uint64_t k = 0; k < K; k += 2) {
            step(b0, b1, k);
            if (k + 1 >= K) break;
            step(b1, b0, k + 1);
        }
    }

    // Slow region: chunks after the last whole unit, plus the short tail chunk, one
    // lane per chunk (at most a unit's worth, so a handful of lanes).
    const uint64_t nfull = a.len / BPC;
    const uint64_t first_slow = nunits * kChunksPerUnit;
    const uint64_t nslow = nfull - first_slow + (a.len % BPC ? 1 : 0);
    const uint64_t gtid = uint64_t(blockIdx.x) * kBlockThreads + threadIdx.x;
    if (gtid < nslow) {
        const uint64_t chunk = first_slow + gtid;
        const uint32_t sz = chunk < nfull ? uint32_t(BPC) : uint32_t(a.len % BPC);
        const uint32_t c = ~crc_run_lines(t, 0xFFFFFFFFu, a.data + chunk * BPC, sz);
        if constexpr (VERIFY) {
            if ((sz == uint32_t(BPC) || a.check_short_tail) && load_be32(a.crc_be + 4 * chunk, crc_al4) != c)
                atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
        } else {
            store_be32(a.out_be + 4 * chunk, c, crc_al4);
        }
    }
}

// ---- wave kernel: round kernel + LDS nibble fold + optional 2-chain interleave ----
//
// Same rounds/regroup as crc32c_rounds_kernel, two changes:
//  * the lane fold M_j (advance over (G-1-j)*64 bytes) reads lane-specific nibble
//    tables kept in the last 32 KiB of LDS (word ((k*16+e)*64 + lane): each lane its
//    own bank): 8 lookups + ~19 VALU instead of a 32-column product in VGPRs;
//  * PAIR = 2 consumes two rounds per step with their lookup chains software-
//    pipelined (sched_barrier-pinned phases: chain 1's 4 reads fly while chain 0
//    folds its previous 4), so each lane keeps two LDS round trips in flight.
constexpr int kFoldLdsOff = kLdsBytes;                  // byte offset of the nibble tables
constexpr int kLdsBytesWave = kLdsBytes + 32 * 1024;    // 160 KiB: the whole CU LDS

struct NibFold {
    const uint8_t *f;  // lds + kFoldLdsOff + lane*4
    __device__ __forceinline__ explicit NibFold(const uint32_t *lds)
        : f(reinterpret_cast<const uint8_t *>(lds) + kFoldLdsOff + 4 * (threadIdx.x & 63)) {}
    __device__ __forceinline__ uint32_t ld(uint32_t off) const {
        return *reinterpret_cast<const uint32_t *>(f + off);
    }
    __device__ __forceinline__ uint32_t apply(uint32_t x) const {
        const uint32_t a0 = ld(((x << 8) & 0xF00u) + 0 * 4096);
        const uint32_t a1 = ld(((x << 4) & 0xF00u) + 1 * 4096);
        const uint32_t a2 = ld((x & 0xF00u) + 2 * 4096);
        const uint32_t a3 = ld(((x >> 4) & 0xF00u) + 3 * 4096);
        const uint32_t a4 = ld(((x >> 8) & 0xF00u) + 4 * 4096);
        const uint32_t a5 = ld(((x >> 12) & 0xF00u) + 5 * 4096);
        const uint32_t a6 = ld(((x >> 16) & 0xF00u) + 6 * 4096);
        const uint32_t a7 = ld(((x >> 20) & 0xF00u) + 7 * 4096);
        return xor3(xor3(a0, a1, a2), xor3(a3, a4, a5), a6 ^ a7);
    }
    // Same product. Spreading the nibbles over bytes lets ONE v_perm build each address:
    // byte 0 = lane*4 and byte 2 = the fold region (from the lane base), byte 1 = nibble;
    // the table (k*4096) rides in the ds_read offset.
    __device__ __forceinline__ uint32_t apply_perm(uint32_t x) const {
        const uint32_t lo = x & 0x0F0F0F0Fu, hi = (x >> 4) & 0x0F0F0F0Fu;
        const uint32_t fb = kFoldLdsOff + 4 * (threadIdx.x & 63);
        const uint8_t *l0 = f - fb;  // LDS base
        auto at = [&](uint32_t src, uint32_t byte, int k) {
            const uint32_t addr = __builtin_amdgcn_perm(src, fb, 0x0C020000u | ((4u + byte) << 8));
            return *reinterpret_cast<const uint32_t *>(l0 + addr + k * 4096);
        };
        const uint32_t a0 = at(lo, 0, 0), a1 = at(hi, 0, 1), a2 = at(lo, 1, 2), a3 = at(hi, 1, 3);
        const uint32_t a4 = at(lo, 2, 4), a5 = at(hi, 2, 5), a6 = at(lo, 3, 6), a7 = at(hi, 3, 7);
        return xor3(xor3(a0, a1, a2), xor3(a3, a4, a5), a6 ^ a7);
    }
};

// The 4 table reads of one word step, and their fold into the next state.
struct Look {
    uint32_t v[4];
};
__device__ __forceinline__ Look lookups(const Lut &t, uint32_t x) {
    Look l;
    l.v[0] = t.at<0>(3, x);
    l.v[1] = t.at<1>(2, x);
    l.v[2] = t.at<2>(1, x);
    l.v[3] = t.at<3>(0, x);
    return l;
}
// Diagnostic (kOptFakeLut): the same v_perm address math with a VALU op where the
// ds_read would be (no LDS traffic, wrong results).
__device__ __forceinline__ Look fake_lookups(const Lut &t, uint32_t x) {
    Look l;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t addr = __builtin_amdgcn_perm(x, t.base[i], 0x0C020000u | ((7u - i) << 8));
        l.v[i] = __builtin_amdgcn_alignbit(addr, addr, 7 + i);
    }
    return l;
}
__device__ __forceinline__ uint32_t combine(const Look &l, uint32_t next) {
    return xor3(xor3(l.v[0], l.v[1], l.v[2]), l.v[3], next);
}

constexpr int kPoolFoldOff = kLdsBytes;                 // 128 KiB
constexpr int kPoolCtrOff = kLdsBytes + 16 * 1024;      // 144 KiB
constexpr int kPoolLdsBytes = kPoolCtrOff + 16;

// OFF: byte offset of the image; its 64 KiB part rides in address byte 2 (the nibble owns
// byte 1), the rest in the ds_read immediate offset
template <int OFF = kPoolFoldOff>
__device__ __forceinline__ uint32_t fold_half(const uint8_t *lds, uint32_t x) {
    const uint32_t lo = x & 0x0F0F0F0Fu, hi = (x >> 4) & 0x0F0F0F0Fu;
    const uint32_t fb = (OFF & ~0xFFFF) + 4 * (threadIdx.x & 31);
    auto at = [&](uint32_t src, uint32_t byte, int off) {
        const uint32_t addr = __builtin_amdgcn_perm(src, fb, 0x0C020000u | ((4u + byte) << 8));
        return *reinterpret_cast<const uint32_t *>(lds + addr + (OFF & 0xFFFF) + off);
    };
    const uint32_t a0 = at(lo, 0, 0), a1 = at(hi, 0, 128), a2 = at(lo, 1, 4096), a3 = at(hi, 1, 4096 + 128);
    const uint32_t a4 = at(lo, 2, 8192), a5 = at(hi, 2, 8192 + 128), a6 = at(lo, 3, 12288);
    const uint32_t a7 = at(hi, 3, 12288 + 128);
    return xor3(xor3(a0, a1, a2), xor3(a3, a4, a5), a6 ^ a7);
}

// OPT bits (experiments kept for A/B, tools/ab.py):
//  kOptFillFirst: every wave of the workgroup issues its table/fold-image loads before any
//    wave issues data loads (s_barrier between). The CU returns loads in order, so a table
//    load queued behind other waves' HBM rounds waits for them at the CU's HBM share.
constexpr int kOptFillFirst = 1;
//  kOptFillWait: the LDS fill completes (table loads returned) before any data load issues.
constexpr int kOptFillWait = 2;
//  kOptNoHbm (diagnostic only, wrong results): every round reads the cache-resident table
//    image instead of the block, so the launch runs at the kernel's compute/LDS rate.
constexpr int kOptNoHbm = 4;
//  kOptNoFill / kOptNoMath (diagnostics only, wrong results): skip the LDS table fill
//    (tables are garbage) / replace the table CRC of a round by an xor of its words.
constexpr int kOptNoFill = 8;
constexpr int kOptNoMath = 16;
//  kOptNibPerm: fold addresses by v_perm from the nibble-spread state (x & 0x0F0F0F0F,
//    (x >> 4) & 0x0F0F0F0F): 11 VALU for the 8 addresses instead of 22.
constexpr int kOptNibPerm = 32;
//  kOptPf2: (PAIR 2) loads run two steps ahead of the lookups (6 round buffers, not 4).
constexpr int kOptPf2 = 64;
//  kOptWantBuf: (verify) stored CRC words through a buffer resource on the wave-uniform
//    word base (lane offset the only VGPR): no 64-bit VGPR address temporaries, which the
//    allocator can put on registers of in-flight round loads (a vmcnt(0) drain per step).
constexpr int kOptWantBuf = 128;
//  kOptLate: the step's prefetch issues after its own rounds arrived (0-8 KiB in flight
//    per wave instead of 8-16). kOptSplit: the second prefetch round issues mid-step.
constexpr int kOptLate = 256;
constexpr int kOptSplit = 512;
//  kOptFakeLut (diagnostic only, wrong results): table reads replaced by a VALU op.
constexpr int kOptFakeLut = 2048;
//  kOptSlotRegion: the 16 wave slots of a workgroup own 16 contiguous regions of the
//    block; the 256 waves of one slot walk their region together (workgroup-interleaved
//    4 KiB rounds). The SIMD arbiter favours older waves, so slots drift apart: with the
//    round-robin mapping the in-flight requests then scatter over the whole block, with
//    regions each slot's requests stay in one compact window.
constexpr int kOptSlotRegion = 4096;
//  kOptVgprFold: the lane fold as a 32-column GF(2) product in VGPRs (gf2_apply4, 64 VALU)
//    instead of 8 nibble-table reads: trades LDS returns for VALU (§5.0).
constexpr int kOptVgprFold = 8192;
//  kOptNtStore: (compute) the CRC words go out as non-temporal stores.
constexpr int kOptNtStore = 16384;
//  kOptLeanFill: each thread loads ONE slice-table word and writes its 32 copies (4 KiB of
//    L2 reads per CU instead of 32 KiB); for bpc <= 2048 the fold image is the half-size
//    one of the pool kernel (16 KiB, one v_perm per fold address).
constexpr int kOptLeanFill = 32768;
//  kOptNoStore (diagnostic only, wrong results): compute mode skips its CRC-word stores.
constexpr int kOptNoStore = 65536;
//  kOptLineStore: (compute, bpc 512) a wave takes 4 consecutive rounds (16 KiB, 32 chunks)
//    per visit and stores their 32 CRC words as ONE full 128-B line from lanes 0..31, instead
//    of one 32-B partial line per round. The words are transposed into lane order by one
//    ds_bpermute per round.
constexpr int kOptLineStore = 131072;
//  kOptHoldStore: (compute, bpc 512) batch the CRC-word stores in time: a wave transposes
//    each 8 rounds' 64 words into one VGPR (lane 8r + c = chunk c of round r) and keeps up
//    to 8 such VGPRs (64 rounds), storing them only when full and at the end of its stream.
constexpr int kOptHoldStore = 262144;
//  kOptPitch: the rounds of a packet stream at a constant pitch (ChunkLaunch::pitch): round u
//    is round u & (upp - 1) of packet u >> upp_log2, so a wave walks packets with two SALU ops
//    per round more than a contiguous block, and the wire layout's per-packet CRC regions are
//    read/written in place. Result keys are (packet << 32) | chunk. The packet API's constant-
//    pitch streams (reader arenas, resident packet rings) take this instead of the segmented
//    kernel.
constexpr int kOptPitch = 524288;
//  kOptHead2: (PAIR 2, PF 1) the prologue loads the first TWO steps' rounds (4 rounds) before
//    the LDS fill, and the first step issues no prefetch: the step-1 loads no longer wait for
//    the fill barrier, while the steady-state depth (one step ahead) is unchanged.
constexpr int kOptHead2 = 1048576;
//  kOptFastTail: (PAIR 2, PF 1, G <= 32) a wave's LAST step runs each round as two 32-byte
//    chains per lane (4 chains of 8 word steps instead of 2 of 16): the lookup chain that runs
//    after the wave's last data arrived is half as long. The halves join as
//    x = M_32(x_A) ^ x_B, M_32 = advance over 32 bytes, read from a lane-replicated nibble
//    image in the LDS's last 16 KiB (ChunkLaunch::m32, 8 lookups per round, last step only).
constexpr int kOptFastTail = 2097152;
constexpr int kTailFoldOff = kLdsBytes + 16 * 1024;  // 144 KiB: M_32 nibble image (16 KiB)
//  kOptSkew: uneven work per workgroup for back-to-back overlapped launches. The first half of
//    the workgroups take base + base/4 rounds per wave, the second half base - base/4 (rounds
//    0 .. (base - base/4) * nwaves - 1 round-robin over every wave as usual, the rest
//    round-robin over the heavy waves only). With overlapped launches the CP hands the next
//    launch's first (heavy) workgroups to the CUs that freed first (they ran light ones), so
//    CUs alternate heavy/light and their launch heads — dispatch, fill, first-data latency,
//    when a CU pulls no HBM bytes — no longer line up across the chip.
constexpr int kOptSkew = 8388608;
//  kOptDiagTail (diagnostic only, wrong results): a wave's last step replaces the table CRC by an
//    xor of its words, so the compute that runs after the wave's last data arrived is ~free. The
//    difference to production is what the per-launch tail costs.
constexpr int kOptDiagTail = 16777216;
//  kOptSoloTail: the wave's last two rounds run one after the other as single chains (no
//    interleave), so the first one's lookups overlap the second one's arrival.
constexpr int kOptSoloTail = 33554432;
//  kOptDiagTailLut (diagnostic only, with kOptDiagTail): the last step keeps its 64 lookups per
//    round but drops their dependency chain (independent lookups of the data words): separates
//    the tail's LDS work from its latency.
constexpr int kOptDiagTailLut = 67108864;
//  kOptSoloHalf (with kOptSoloTail): the wave's very last round as two interleaved 32-byte half
//    chains joined in VALU (x = M_32(x_a) ^ x_b): half the dependent lookups after the last data.
constexpr int kOptSoloHalf = 134217728;

template <int BPC, bool VERIFY, int PAIR, bool NT = false, bool BUF = true, bool TRACE = false, bool PRIO = false,
          int OPT = 0>
__global__ __launch_bounds__(kBlockThreads) void crc32c_wave_r2_kernel(ChunkLaunch a,
                                                                    const uint32_t *__restrict__ g_tab,
                                                                    const uint32_t *__restrict__ g_nib) {
    static_assert(BPC <= kRoundBytes, "one-round units only");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytesWave / 4];
    constexpr int G = BPC / 64;
    constexpr int kChunksPerUnit = kRoundBytes / BPC;

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane % G;
    const uint32_t lane_off = 64 * (lane & 15) + 16 * (lane >> 4);
    constexpr bool kPit = (OPT & kOptPitch) != 0;
    const uint64_t nunits = kPit ? ((a.npk - 1) << a.upp_log2) + a.last_len / kRoundBytes : a.len / kRoundBytes;
    // kPit: unit u -> (packet, round in packet); the contiguous case is packet 0 at pitch 0
    const uint64_t umask = (uint64_t(1) << a.upp_log2) - 1;
    const uint64_t cpitch = a.crc_pitch ? a.crc_pitch : a.pitch;  // the words' pitch
    auto unit_data = [&](uint64_t u) -> const uint8_t * {
        if constexpr (kPit) return a.data + (u >> a.upp_log2) * a.pitch + (u & umask) * kRoundBytes;
        return a.data + u * kRoundBytes;
    };
    // the CRC word of chunk c of unit u (stored words when verifying, the output when computing)
    auto word_ptr = [&](uint64_t u, uint32_t c) -> uint8_t * {
        uint8_t *base = VERIFY ? const_cast<uint8_t *>(a.crc_be) : a.out_be;
        if constexpr (kPit) return base + (u >> a.upp_log2) * cpitch + 4 * ((u & umask) * kChunksPerUnit + c);
        return base + 4 * (u * kChunksPerUnit + c);
    };
    auto key_of = [&](uint64_t u, uint32_t c) -> uint64_t {
        if constexpr (kPit) return ((u >> a.upp_log2) << 32) | ((u & umask) * kChunksPerUnit + c);
        return a.chunk_base + u * kChunksPerUnit + c;
    };
    const uint64_t nwaves = uint64_t(gridDim.x) * kWavesPerBlock;
    // wave-uniform by construction; readfirstlane makes that provable to the compiler so
    // the end-of-stream prefetch guards below are scalar branches, not exec masks
    const uint64_t wave = uint64_t(blockIdx.x) * kWavesPerBlock +
                          __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // this wave's rounds: unit first + k * stride for k < K
    uint64_t first = wave, stride = nwaves, K;
    constexpr bool kLine = !VERIFY && (OPT & kOptLineStore) != 0 && G == 8 && PAIR == 2 && (OPT & kOptPf2) == 0;
    // kLine: round k of the wave is unit 4 * (first + (k >> 2) * stride) + (k & 3)
    auto unit_of = [&](uint64_t k) -> uint64_t {
        if constexpr (kLine) return 4 * (first + (k >> 2) * stride) + (k & 3);
        return first + k * stride;
    };
    if constexpr (kLine) {
        const uint64_t nsup = (nunits + 3) / 4;
        K = wave < nsup ? 4 * ((nsup - wave + nwaves - 1) / nwaves) : 0;
    } else if constexpr ((OPT & kOptSlotRegion) != 0) {
        const uint64_t slot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const uint64_t R = (nunits + kWavesPerBlock - 1) / kWavesPerBlock;
        const uint64_t lo = slot * R, hi = lo + R < nunits ? lo + R : nunits;
        first = lo + blockIdx.x;
        stride = gridDim.x;
        K = first < hi ? (hi - first + stride - 1) / stride : 0;
    } else {
        K = wave < nunits ? (nunits - wave + nwaves - 1) / nwaves : 0;
    }
    // kOptSkew geometry (even base only; otherwise the plain round-robin above)
    constexpr bool kSkewOpt = (OPT & kOptSkew) != 0 && !kLine && (OPT & kOptSlotRegion) == 0;
    const uint64_t sk_base = kSkewOpt ? nunits / nwaves : 0;
    const bool skew = kSkewOpt && nunits % nwaves == 0 && sk_base >= 4 && sk_base % 4 == 0 && gridDim.x % 2 == 0;
    const uint64_t sk_light = sk_base - sk_base / 4, sk_half = nwaves / 2;
    if (skew) K = wave < sk_half ? sk_base + sk_base / 4 : sk_light;
    // unit of the wave's round k
    auto uk = [&](uint64_t k) -> uint64_t {
        if constexpr (kSkewOpt) {
            if (skew && k >= sk_light) return sk_light * nwaves + wave + (k - sk_light) * sk_half;
        }
        return first + k * stride;
    };
    // Prefetches past the wave's last round stay unconditional (a branch around them
    // makes the waitcnt pass drain every load at the loop head) but read the 4 KiB slice
    // table image instead: cache-resident, so they cost no HBM bytes (re-reading data
    // would, since the non-temporal stream is not kept in L2).
    auto round_ptr = [&](uint64_t k) -> const uint8_t * {
        if constexpr ((OPT & kOptNoHbm) != 0) return reinterpret_cast<const uint8_t *>(g_tab);
        if constexpr (kLine) {
            // the wave's last visit may hold fewer than 4 rounds
            const uint64_t u = unit_of(k);
            return k < K && u < nunits ? a.data + u * kRoundBytes : reinterpret_cast<const uint8_t *>(g_tab);
        }
        return k < K ? unit_data(uk(k)) : reinterpret_cast<const uint8_t *>(g_tab);
    };

    // TRACE (variant 13): lane 0 of each wave stamps entry, post-fill, post-first-step
    // and end of the main loop with the device-wide 100 MHz counter
    uint64_t *tr = TRACE ? a.trace + 4 * wave : nullptr;
    auto stamp = [&](int i) {
        if constexpr (TRACE) {
            const uint64_t t = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) tr[i] = t;
        }
    };
    stamp(0);
    // table + nibble-image words, then the first round(s), then the LDS fill
    constexpr bool kLean = (OPT & kOptLeanFill) != 0;
    // the half-size fold image needs lanes l and l + 32 to share fold tables (G <= 32)
    constexpr bool kHalfFold = kLean && G <= 32;
    uint32_t tv[kLean ? 1 : kFillPerThread];
    u32x4 n0, n1;
    constexpr bool kFastTail = (OPT & kOptFastTail) != 0 && kLean && G <= 32 && PAIR == 2 && (OPT & (kOptPf2 | kOptHead2)) == 0;
    uint32_t m32w = 0;  // kFastTail: this thread's word of the M_32 nibble image
    if constexpr (kLean) {
        const uint32_t t = threadIdx.x;
        tv[0] = g_tab[t];  // slice t >> 8, entry t & 255
        if constexpr (kHalfFold) {
            const uint32_t fk = 2 * (t >> 8) + ((t >> 3) & 1), fe = (t >> 4) & 15, fc = 4 * (t & 7);
            n0 = *reinterpret_cast<const u32x4 *>(g_nib + (fk * 16 + fe) * 64 + fc);
            if constexpr (kFastTail) m32w = a.m32[fk * 16 + fe];
        } else {
            n0 = *reinterpret_cast<const u32x4 *>(g_nib + 8 * threadIdx.x);
            n1 = *reinterpret_cast<const u32x4 *>(g_nib + 8 * threadIdx.x + 4);
        }
    } else {
        fetch_tables(tv, g_tab);
        n0 = *reinterpret_cast<const u32x4 *>(g_nib + 8 * threadIdx.x);
        n1 = *reinterpret_cast<const u32x4 *>(g_nib + 8 * threadIdx.x + 4);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((OPT & kOptFillFirst) != 0) asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    auto fill = [&]() {
        if constexpr ((OPT & kOptNoFill) != 0) return;
        if constexpr (kLean) {
            // 32 copies of this thread's entry: 8 x b128, rotated by thread so 8 neighbouring
            // threads (consecutive entries, 256 B apart) hit 8 different bank groups
            const uint32_t t = threadIdx.x, slice = t >> 8, entry = t & 255;
            u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
            const uint32_t slot0 = ((slice >> 1) << 16 | entry << 8 | (slice & 1) << 7) / 16;
#pragma unroll
            for (int r = 0; r < 8; ++r) l4[slot0 + ((r + t) & 7)] = u32x4{tv[0], tv[0], tv[0], tv[0]};
            if constexpr (kHalfFold) {
                reinterpret_cast<u32x4 *>(lds + kPoolFoldOff / 4)[t] = n0;
                if constexpr (kFastTail) reinterpret_cast<u32x4 *>(lds + kTailFoldOff / 4)[t] = u32x4{m32w, m32w, m32w, m32w};
            } else {
                u32x4 *dst = reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(lds) + kFoldLdsOff) + 2 * t;
                dst[0] = n0;
                dst[1] = n1;
            }
        } else {
            store_tables(lds, tv);
            u32x4 *dst = reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(lds) + kFoldLdsOff) + 2 * threadIdx.x;
            dst[0] = n0;
            dst[1] = n1;
        }
        lds_barrier();
    };
    if constexpr ((OPT & kOptFillWait) != 0) fill();
    __builtin_amdgcn_sched_barrier(0);
    constexpr bool kHead2 = (OPT & kOptHead2) != 0 && PAIR == 2 && (OPT & kOptPf2) == 0;
    constexpr int kPro = ((OPT & kOptPf2) != 0 && PAIR == 2) || kHead2 ? 4 : PAIR;  // rounds loaded before the loop
    Round b[kPro == 4 && !kHead2 ? 6 : 2 * PAIR];
#pragma unroll
    for (int i = 0; i < kPro; ++i) {
        load_any<NT, BUF>(b[i], round_ptr(i), lane_off);
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr ((OPT & kOptFillWait) == 0) fill();
    stamp(1);
    const Lut t(lds);
    const NibFold nf(lds);
    const uint32_t init = j == 0 ? 0xFFFFFFFFu : 0u;
    uint32_t col[32];
    if constexpr ((OPT & kOptVgprFold) != 0) {
        constexpr int set = G == 8 ? 0 : G == 16 ? 1 : G == 32 ? 2 : 3;
        constexpr int kFoldOff[4] = {0, 8, 24, 56};
        const uint32_t *g_fold = g_nib - kFoldWords - set * kFoldNibbleWords;
#pragma unroll
        for (int i = 0; i < 32; ++i) col[i] = g_fold[(kFoldOff[set] + j) * 32 + i];
    }
    auto fold = [&](uint32_t x) -> uint32_t {
        if constexpr (kHalfFold) return fold_half(reinterpret_cast<const uint8_t *>(lds), x);
        if constexpr ((OPT & kOptVgprFold) != 0) return gf2_apply4(col, x);
        if constexpr ((OPT & kOptNibPerm) != 0) return nf.apply_perm(x);
        return nf.apply(x);
    };

    auto want_of = [&](uint64_t k) -> uint32_t {
        if constexpr (VERIFY) {
            const uint64_t kk = k < K ? k : K - 1;
            if constexpr ((OPT & kOptWantBuf) != 0) {
                const uint64_t b = reinterpret_cast<uint64_t>(a.crc_be + 4 * (first + kk * stride) * kChunksPerUnit);
                const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(b));
                const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(b >> 32));
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    reinterpret_cast<void *>((uint64_t(hi) << 32) | lo), 0, 4 * kChunksPerUnit, 0x00020000);
                return __builtin_amdgcn_raw_buffer_load_b32(rs, 4 * (lane / G), 0, 0);
            }
            return *reinterpret_cast<const uint32_t *>(word_ptr(uk(kk), lane / G));
        }
        return 0;
    };
    uint32_t line = 0;  // kLine: lane q (< 32) collects word q of the visit's 32 chunks
    constexpr bool kHold = !VERIFY && !kLine && (OPT & kOptHoldStore) != 0 && G == 8 &&
                           (OPT & kOptSlotRegion) == 0;
    uint32_t hold[kHold ? 8 : 1];  // hold[i] = octet hold_base + nheld - 1 - i
    uint32_t nheld = 0;
    uint64_t hold_base = 0;
    auto flush = [&]() {
#pragma unroll
        for (int i = 0; i < (kHold ? 8 : 0); ++i) {
            if (uint32_t(i) < nheld) {
                const uint64_t k = 8 * (hold_base + nheld - 1 - i) + (lane >> 3);
                if (k < K)
                    *reinterpret_cast<uint32_t *>(word_ptr(uk(k), lane & 7)) =
                        __builtin_bswap32(~hold[i]);
            }
        }
        hold_base += nheld;
        nheld = 0;
    };
    auto finish = [&](uint64_t k, uint32_t y, uint32_t want) {
        if constexpr (kHold) {
            if (k >= K) return;
            const uint32_t r = uint32_t(k & 7);
            const uint32_t v = uint32_t(__builtin_amdgcn_ds_bpermute(int(32 * (lane & 7)), int(y)));
            line = (lane >> 3) == r ? v : line;
            if (r == 7 || k + 1 == K) {
#pragma unroll
                for (int i = (kHold ? 7 : 0); i > 0; --i) hold[i] = hold[i - 1];
                hold[0] = line;
                if (++nheld == 8) flush();
            }
            return;
        }
        if constexpr (kLine) {
            // every lane of group c holds chunk c's state (group_xor is a butterfly); lane
            // 8r + c takes chunk c of round r
            const uint32_t r = uint32_t(k & 3);
            const uint32_t v = uint32_t(__builtin_amdgcn_ds_bpermute(int(32 * (lane & 7)), int(y)));
            line = (lane >> 3) == r ? v : line;
            if (r == 3) {
                const uint64_t u0 = unit_of(k - 3);
                if (lane < 32 && u0 + (lane >> 3) < nunits)
                    *reinterpret_cast<uint32_t *>(a.out_be + 4 * (u0 * kChunksPerUnit + lane)) = __builtin_bswap32(~line);
            }
            return;
        }
        if (k >= K || j != 0) return;
        const uint64_t u = uk(k);
        const uint32_t c = ~y;
        if constexpr (VERIFY) {
            const bool bad = (OPT & (kOptNoHbm | kOptNoFill | kOptNoMath | kOptFakeLut | kOptDiagTail)) != 0
                                   ? __builtin_bswap32(want) == ~c
                                   : __builtin_bswap32(want) != c;
            if (bad) atomicMax(a.result, ~(unsigned long long)key_of(u, lane / G));
        } else if constexpr ((OPT & kOptNoStore) != 0) {
            if (c == 0x9E3779B9u) *reinterpret_cast<uint32_t *>(word_ptr(u, lane / G)) = c;
        } else if constexpr ((OPT & kOptNtStore) != 0) {
            __builtin_nontemporal_store(__builtin_bswap32(c), reinterpret_cast<uint32_t *>(word_ptr(u, lane / G)));
        } else {
            *reinterpret_cast<uint32_t *>(word_ptr(u, lane / G)) = __builtin_bswap32(c);
        }
    };
    // word i (0..15) of the lane's 64-byte segment after regroup
    auto word = [](const Round &r, int i) -> uint32_t { return r.w[i >> 2][i & 3]; };

    if constexpr (PAIR == 1) {
        auto step = [&](Round &cur, Round &pf, uint64_t k) {
            const uint32_t w = want_of(k);
            load_any<NT, BUF>(pf, round_ptr(k + 1), lane_off);
            __builtin_amdgcn_sched_barrier(0);
            regroup(cur);
            uint32_t x = init ^ word(cur, 0);
#pragma unroll
            for (int i = 0; i < 16; ++i) x = combine(lookups(t, x), i < 15 ? word(cur, i < 15 ? i + 1 : 15) : 0u);
            finish(k, group_xor<G>(nf.apply(x)), w);
        };
        for (uint64_t k = 0; k < K; k += 2) {
            step(b[0], b[1], k);
            if (k + 1 >= K) break;
            step(b[1], b[0], k + 1);
        }
    } else {
        constexpr int PF = (OPT & kOptPf2) != 0 ? 2 : 1;  // steps of loads in flight
        auto step = [&](Round &c0, Round &c1, Round &p0, Round &p1, uint64_t k, auto do_pf, auto do_math) {
            constexpr bool kPf = decltype(do_pf)::value;
            const uint32_t w0 = want_of(k), w1 = want_of(k + 1);
            constexpr bool kLate = (OPT & kOptLate) != 0 || !kPf, kSplit = (OPT & kOptSplit) != 0;
            if constexpr (!kLate) load_any<NT, BUF>(p0, round_ptr(k + 2 * PF), lane_off);
            if constexpr (!kLate && !kSplit) load_any<NT, BUF>(p1, round_ptr(k + 2 * PF + 1), lane_off);
            __builtin_amdgcn_sched_barrier(0);
            regroup(c0);
            regroup(c1);
            if constexpr (kLate && kPf) {
                __builtin_amdgcn_sched_barrier(0);
                load_any<NT, BUF>(p0, round_ptr(k + 2 * PF), lane_off);
                load_any<NT, BUF>(p1, round_ptr(k + 2 * PF + 1), lane_off);
                __builtin_amdgcn_sched_barrier(0);
            }
            uint32_t x0 = init ^ word(c0, 0), x1 = init ^ word(c1, 0);
            if constexpr ((OPT & kOptDiagTailLut) != 0 && !decltype(do_math)::value) {
                // diagnostic: the same 64 lookups per round with no dependency chain
                uint32_t a0 = 0, a1 = 0;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    a0 ^= combine(lookups(t, word(c0, i)), 0u);
                    a1 ^= combine(lookups(t, word(c1, i)), 0u);
                }
                x0 ^= a0;
                x1 ^= a1;
            } else if constexpr ((OPT & kOptNoMath) != 0 || !decltype(do_math)::value) {
#pragma unroll
                for (int i = 1; i < 16; ++i) {
                    x0 ^= word(c0, i);
                    x1 ^= word(c1, i);
                }
            } else {
            auto lookups = [&](const Lut &t, uint32_t x) {
                if constexpr ((OPT & kOptFakeLut) != 0) return fake_lookups(t, x);
                return ::hdfs3crc::lookups(t, x);
            };
            Look l0 = lookups(t, x0), l1;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if constexpr (kSplit && !kLate && kPf) {
                    if (i == 8) {
                        load_any<NT, BUF>(p1, round_ptr(k + 2 * PF + 1), lane_off);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                l1 = lookups(t, x1);
                __builtin_amdgcn_sched_barrier(0);
                x0 = combine(l0, i < 15 ? word(c0, i < 15 ? i + 1 : 15) : 0u);
                __builtin_amdgcn_sched_barrier(0);
                if (i < 15) l0 = lookups(t, x0);
                __builtin_amdgcn_sched_barrier(0);
                x1 = combine(l1, i < 15 ? word(c1, i < 15 ? i + 1 : 15) : 0u);
                __builtin_amdgcn_sched_barrier(0);
            }
            }
            const uint32_t y0 = group_xor<G>(fold(x0));
            const uint32_t y1 = group_xor<G>(fold(x1));
            finish(k, y0, w0);
            finish(k + 1, y1, w1);
        };
        // PRIO: the SIMD arbiter favours older waves, so with equal work the 4 waves of a
        // SIMD finish staggered and the last ones run alone, too few to keep the CU's
        // share of HBM busy (tools/wave_trace.py). Priority by work remaining (quartiles,
        // s_setprio 3..0) lets lagging waves catch up so the CU drains together.
        auto prio = [&](uint64_t k) {
            if constexpr (PRIO) {
                const uint64_t left = K - k;  // rounds still to consume, incl. this step
                const uint32_t p = uint32_t(left * 4 > 3 * K ? 3 : left * 4 > 2 * K ? 2 : left * 4 > K ? 1 : 0);
                switch (p) {  // s_setprio takes an immediate
                case 3: __builtin_amdgcn_s_setprio(3); break;
                case 2: __builtin_amdgcn_s_setprio(2); break;
                case 1: __builtin_amdgcn_s_setprio(1); break;
                default: __builtin_amdgcn_s_setprio(0); break;
                }
            }
        };
        using pf_on = std::integral_constant<bool, true>;
        using pf_off = std::integral_constant<bool, false>;
        using math_on = std::integral_constant<bool, true>;
        using math_off = std::integral_constant<bool, false>;
        // kFastTail: the wave's last step, no prefetch, four half-round chains
        auto tail = [&](Round &c0, Round &c1, uint64_t k) {
            const uint32_t w0 = want_of(k), w1 = want_of(k + 1);
            __builtin_amdgcn_sched_barrier(0);
            regroup(c0);
            regroup(c1);
            uint32_t xa0 = init ^ word(c0, 0), xb0 = word(c0, 8), xa1 = init ^ word(c1, 0), xb1 = word(c1, 8);
            Look la0 = lookups(t, xa0), lb0 = lookups(t, xb0), la1, lb1;
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                la1 = lookups(t, xa1);
                lb1 = lookups(t, xb1);
                __builtin_amdgcn_sched_barrier(0);
                xa0 = combine(la0, i < 7 ? word(c0, i < 7 ? i + 1 : 7) : 0u);
                xb0 = combine(lb0, i < 7 ? word(c0, i < 7 ? i + 9 : 15) : 0u);
                __builtin_amdgcn_sched_barrier(0);
                if (i < 7) {
                    la0 = lookups(t, xa0);
                    lb0 = lookups(t, xb0);
                }
                __builtin_amdgcn_sched_barrier(0);
                xa1 = combine(la1, i < 7 ? word(c1, i < 7 ? i + 1 : 7) : 0u);
                xb1 = combine(lb1, i < 7 ? word(c1, i < 7 ? i + 9 : 15) : 0u);
                __builtin_amdgcn_sched_barrier(0);
            }
            const uint8_t *l8 = reinterpret_cast<const uint8_t *>(lds);
            const uint32_t x0 = fold_half<kTailFoldOff>(l8, xa0) ^ xb0;
            const uint32_t x1 = fold_half<kTailFoldOff>(l8, xa1) ^ xb1;
            finish(k, group_xor<G>(fold(x0)), w0);
            finish(k + 1, group_xor<G>(fold(x1)), w1);
        };
        if constexpr (kFastTail) {
            for (uint64_t k = 0; k < K; k += 4) {
                if (k + 2 >= K) {
                    tail(b[0], b[1], k);
                    break;
                }
                step(b[0], b[1], b[2], b[3], k, pf_on{}, math_on{});
                if (k == 0) stamp(2);
                if (k + 4 >= K) {
                    tail(b[2], b[3], k + 2);
                    break;
                }
                step(b[2], b[3], b[0], b[1], k + 2, pf_on{}, math_on{});
            }
        } else if constexpr (kHead2) {
            // step 0 consumes b0/b1 without a prefetch (b2/b3 already hold step 1), then the
            // usual one-step-ahead rotation from step 1 on
            if (K > 0) {
                step(b[0], b[1], b[2], b[3], 0, pf_off{}, math_on{});
                stamp(2);
            }
            for (uint64_t k = 2; k < K; k += 4) {
                step(b[2], b[3], b[0], b[1], k, pf_on{}, math_on{});
                if (k + 2 >= K) break;
                step(b[0], b[1], b[2], b[3], k + 2, pf_on{}, math_on{});
            }
        } else if constexpr (PF == 1 && (OPT & kOptSoloTail) != 0) {
            // the wave's last two rounds one after the other, each as a single chain: round k's
            // chain runs while round k + 1 is still arriving, and only one round's lookups
            // remain once the wave's last data has landed
            auto solo = [&](Round &c, uint64_t k) {
                const uint32_t w = want_of(k);
                __builtin_amdgcn_sched_barrier(0);
                regroup(c);
                uint32_t x = init ^ word(c, 0);
#pragma unroll
                for (int i = 0; i < 16; ++i) x = combine(lookups(t, x), i < 15 ? word(c, i < 15 ? i + 1 : 15) : 0u);
                finish(k, group_xor<G>(fold(x)), w);
            };
            // kOptSoloHalf: the very last round as two 32-byte half chains, interleaved, joined by
            // x = M_32(x_a) ^ x_b with M_32 as a 32-column GF(2) product in VALU (columns read once
            // from the ctx's M_32 nibble image: word (i / 4) * 16 + (1 << i % 4) = M_32(1 << i))
            auto solo_last = [&](Round &c, uint64_t k) {
                if constexpr ((OPT & kOptSoloHalf) != 0) {
                    // wave-uniform columns, loaded here so they are live only in the last round
                    uint32_t m32c[32];
#pragma unroll
                    for (int i = 0; i < 32; ++i)
                        m32c[i] = __builtin_amdgcn_readfirstlane(a.m32[(i >> 2) * 16 + (1u << (i & 3))]);
                    const uint32_t w = want_of(k);
                    __builtin_amdgcn_sched_barrier(0);
                    regroup(c);
                    uint32_t xa = init ^ word(c, 0), xb = word(c, 8);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const Look la = lookups(t, xa), lb = lookups(t, xb);
                        xa = combine(la, i < 7 ? word(c, i < 7 ? i + 1 : 7) : 0u);
                        xb = combine(lb, i < 7 ? word(c, i < 7 ? i + 9 : 15) : 0u);
                    }
                    finish(k, group_xor<G>(fold(gf2_apply4(m32c, xa) ^ xb)), w);
                } else {
                    solo(c, k);
                }
            };
            for (uint64_t k = 0; k < K; k += 4) {
                if (k + 2 >= K) {
                    if (k + 1 < K) {
                        solo(b[0], k);
                        solo_last(b[1], k + 1);
                    } else {
                        solo_last(b[0], k);
                    }
                    break;
                }
                step(b[0], b[1], b[2], b[3], k, pf_on{}, math_on{});
                if (k + 4 >= K) {
                    if (k + 3 < K) {
                        solo(b[2], k + 2);
                        solo_last(b[3], k + 3);
                    } else {
                        solo_last(b[2], k + 2);
                    }
                    break;
                }
                step(b[2], b[3], b[0], b[1], k + 2, pf_on{}, math_on{});
            }
        } else if constexpr (PF == 1 && (OPT & kOptDiagTail) != 0) {
            // diagnostic: a wave's last step skips the table CRC (wrong results on purpose)
            for (uint64_t k = 0; k < K; k += 4) {
                if (k + 2 >= K) {
                    step(b[0], b[1], b[2], b[3], k, pf_on{}, math_off{});
                    break;
                }
                step(b[0], b[1], b[2], b[3], k, pf_on{}, math_on{});
                if (k + 4 >= K) {
                    step(b[2], b[3], b[0], b[1], k + 2, pf_on{}, math_off{});
                    break;
                }
                step(b[2], b[3], b[0], b[1], k + 2, pf_on{}, math_on{});
            }
        } else if constexpr (PF == 1) {
            for (uint64_t k = 0; k < K; k += 4) {
                prio(k);
                step(b[0], b[1], b[2], b[3], k, pf_on{}, math_on{});
                if (k == 0) stamp(2);
                if (k + 2 >= K) break;
                prio(k + 2);
                step(b[2], b[3], b[0], b[1], k + 2, pf_on{}, math_on{});
            }
        } else {
            for (uint64_t k = 0; k < K; k += 6) {
                step(b[0], b[1], b[4], b[5], k, pf_on{}, math_on{});
                if (k == 0) stamp(2);
                if (k + 2 >= K) break;
                step(b[2], b[3], b[0], b[1], k + 2, pf_on{}, math_on{});
                if (k + 4 >= K) break;
                step(b[4], b[5], b[2], b[3], k + 4, pf_on{}, math_on{});
            }
        }
    }
    if constexpr (kHold) flush();
    stamp(3);

    // slow region: chunks after the last whole round, plus the short tail chunk (kPit: of the
    // last packet, the only one that may end inside a round)
    const uint64_t len = kPit ? a.last_len : a.len;
    const uint8_t *sdata = kPit ? a.data + (a.npk - 1) * a.pitch : a.data;
    uint8_t *sw = (VERIFY ? const_cast<uint8_t *>(a.crc_be) : a.out_be) + (kPit ? (a.npk - 1) * cpitch : 0);
    const uint64_t skey = kPit ? (a.npk - 1) << 32 : a.chunk_base;
    const uint64_t nfull = len / BPC;
    const uint64_t first_slow = (len / kRoundBytes) * kChunksPerUnit;
    const uint64_t nslow = nfull - first_slow + (len % BPC ? 1 : 0);
    const uint64_t gtid = uint64_t(blockIdx.x) * kBlockThreads + threadIdx.x;
    const bool crc_al4 = (reinterpret_cast<uintptr_t>(sw) & 3u) == 0;
    if (gtid < nslow) {
        const uint64_t chunk = first_slow + gtid;
        const uint32_t sz = chunk < nfull ? uint32_t(BPC) : uint32_t(len % BPC);
        const uint32_t c = ~crc_run_lines(t, 0xFFFFFFFFu, sdata + chunk * BPC, sz);
        if constexpr (VERIFY) {
            if ((sz == uint32_t(BPC) || a.check_short_tail) && load_be32(sw + 4 * chunk, crc_al4) != c)
                atomicMax(a.result, ~(unsigned long long)(skey + chunk));
        } else {
            store_be32(sw + 4 * chunk, c, crc_al4);
        }
    }
}

// ---- pool kernel: the wave kernel with per-CU dynamic round pairs (bpc <= 2048) ----
//
// The wave kernel assigns rounds statically (wave w: rounds w, w + W, ...). The SIMD
// arbiter favours older waves, so the 16 waves of a CU drift apart: the oldest finish
// their 8 rounds first and the youngest run their last steps alone, latency-bound, while
// the CU's in-flight reads spread over a wider address window (tools/wave_trace.py).
// Here the rounds of a workgroup form a POOL in address order (16-round segments at the
// round-robin stride W = 16 * grid: unit wg*16 + i % 16 + (i / 16) * W for pool index i),
// and every wave takes the next pair from an LDS counter (ds_add_rtn, lane 0) one step
// ahead of its prefetch: faster waves take more pairs, the CU's reads stay the next
// pairs of the pool, and all waves of a CU end within one step of each other.
//
// LDS: slice tables 128 KiB, then a HALF-size fold image (16 KiB): for G <= 32 lanes l and
// l + 32 hold the same fold tables and never share a ds_read cycle, so 32 columns serve the
// wave. Word (k >> 1) * 1024 + e * 64 + (k & 1) * 32 + (lane & 31) = M_j(e << 4k): the
// nibble sits in address byte 1, so ONE v_perm on the nibble-spread state builds each
// fold address; (k >> 1) * 4096 + (k & 1) * 128 rides in the ds_read offset. Then the
// pool counter.
template <int BPC, bool VERIFY, bool TRACE = false>
__global__ __launch_bounds__(kBlockThreads) void crc32c_pool_kernel(ChunkLaunch a, const uint32_t *__restrict__ g_tab,
                                                                    const uint32_t *__restrict__ g_nib) {
    static_assert(BPC <= 2048 && BPC % 64 == 0, "G <= 32: lanes l and l + 32 share fold tables");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kPoolLdsBytes / 4];
    constexpr int G = BPC / 64;
    constexpr int kChunksPerUnit = kRoundBytes / BPC;
    const uint8_t *lds8 = reinterpret_cast<const uint8_t *>(lds);
    uint32_t *ctr = lds + kPoolCtrOff / 4;  // LDS byte kPoolCtrOff (the array starts at LDS 0)

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane % G;
    const uint32_t lane_off = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint32_t slot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nunits = a.len / kRoundBytes;
    const uint64_t W = uint64_t(gridDim.x) * kWavesPerBlock;
    const uint64_t wg0 = uint64_t(blockIdx.x) * kWavesPerBlock;
    // pool index -> unit (monotone: once a pool index is past the end, so is every later one)
    auto unit_of = [&](uint32_t i) -> uint64_t { return wg0 + (i & 15u) + uint64_t(i >> 4) * W; };
    // past the end, loads stay unconditional but read the cache-resident table image
    auto round_ptr = [&](uint64_t u) -> const uint8_t * {
        return u < nunits ? a.data + u * kRoundBytes : reinterpret_cast<const uint8_t *>(g_tab);
    };

    uint64_t *tr = TRACE ? a.trace + 4 * (wg0 + slot) : nullptr;
    auto stamp = [&](int i) {
        if constexpr (TRACE) {
            const uint64_t t = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) tr[i] = t;
        }
    };
    stamp(0);
    const uint32_t tw = g_tab[threadIdx.x];  // lean fill: one slice-table word per thread
    // half fold image: this thread's 4 LDS words w = 4 * tid
    const uint32_t t = threadIdx.x;
    const uint32_t fk = 2 * (t >> 8) + ((t >> 3) & 1), fe = (t >> 4) & 15, fc = 4 * (t & 7);
    const u32x4 nv = *reinterpret_cast<const u32x4 *>(g_nib + (fk * 16 + fe) * 64 + fc);
    __builtin_amdgcn_sched_barrier(0);
    // the first two pairs are static (pool indices 2 slot and 32 + 2 slot); the counter
    // hands out pairs from 64 on
    uint32_t ic = 2 * slot, in = 32 + 2 * slot;
    Round b[4];
    load_round_buf<true>(b[0], round_ptr(unit_of(ic)), lane_off);
    __builtin_amdgcn_sched_barrier(0);
    load_round_buf<true>(b[1], round_ptr(unit_of(ic + 1)), lane_off);
    __builtin_amdgcn_sched_barrier(0);
    {
        const uint32_t slice = t >> 8, entry = t & 255;
        u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
        const uint32_t slot0 = ((slice >> 1) << 16 | entry << 8 | (slice & 1) << 7) / 16;
#pragma unroll
        for (int r = 0; r < 8; ++r) l4[slot0 + ((r + t) & 7)] = u32x4{tw, tw, tw, tw};
    }
    reinterpret_cast<u32x4 *>(lds + kPoolFoldOff / 4)[t] = nv;
    if (t == 0) *ctr = 64;
    lds_barrier();
    stamp(1);
    const Lut tb(lds);
    const uint32_t init = j == 0 ? 0xFFFFFFFFu : 0u;

    auto want_of = [&](uint64_t u) -> uint32_t {
        if constexpr (VERIFY) {
            const uint64_t uu = u < nunits ? u : nunits - 1;
            const uint64_t base = reinterpret_cast<uint64_t>(a.crc_be + 4 * uu * kChunksPerUnit);
            const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(base));
            const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(base >> 32));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<void *>((uint64_t(hi) << 32) | lo), 0, 4 * kChunksPerUnit, 0x00020000);
            return __builtin_amdgcn_raw_buffer_load_b32(rs, 4 * (lane / G), 0, 0);
        }
        return 0;
    };
    auto finish = [&](uint64_t u, uint32_t y, uint32_t want) {
        if (u >= nunits || j != 0) return;
        const uint64_t chunk = u * kChunksPerUnit + lane / G;
        const uint32_t c = ~y;
        if constexpr (VERIFY) {
            if (__builtin_bswap32(want) != c) atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
        } else {
            *reinterpret_cast<uint32_t *>(a.out_be + 4 * chunk) = __builtin_bswap32(c);
        }
    };
    auto word = [](const Round &r, int i) -> uint32_t { return r.w[i >> 2][i & 3]; };

    uint32_t grab = 0;
    bool first_step = true;
    auto step = [&](Round &c0, Round &c1, Round &p0, Round &p1) {
        const uint64_t u0 = unit_of(ic), u1 = unit_of(ic + 1);
        const uint32_t w0 = want_of(u0), w1 = want_of(u1);
        load_round_buf<true>(p0, round_ptr(unit_of(in)), lane_off);
        load_round_buf<true>(p1, round_ptr(unit_of(in + 1)), lane_off);
        // the pair after next: one LDS atomic by lane 0, issued as asm so the compiler neither
        // spreads it over the wave nor waits for its result here (the step's table reads
        // return after it, so it is long back when `grab` is read at the end of the step)
        if (lane == 0)
            asm volatile("ds_add_rtn_u32 %0, %1, %2" : "=v"(grab) : "v"(kPoolCtrOff), "v"(2u) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        regroup(c0);
        regroup(c1);
        uint32_t x0 = init ^ word(c0, 0), x1 = init ^ word(c1, 0);
        Look l0 = lookups(tb, x0), l1;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            l1 = lookups(tb, x1);
            __builtin_amdgcn_sched_barrier(0);
            x0 = combine(l0, i < 15 ? word(c0, i < 15 ? i + 1 : 15) : 0u);
            __builtin_amdgcn_sched_barrier(0);
            if (i < 15) l0 = lookups(tb, x0);
            __builtin_amdgcn_sched_barrier(0);
            x1 = combine(l1, i < 15 ? word(c1, i < 15 ? i + 1 : 15) : 0u);
            __builtin_amdgcn_sched_barrier(0);
        }
        const uint32_t y0 = group_xor<G>(fold_half(lds8, x0));
        const uint32_t y1 = group_xor<G>(fold_half(lds8, x1));
        finish(u0, y0, w0);
        finish(u1, y1, w1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ic = in;
        in = __builtin_amdgcn_readfirstlane(grab);
        if (first_step) {
            stamp(2);
            first_step = false;
        }
    };
    for (;;) {
        if (unit_of(ic) >= nunits) break;
        step(b[0], b[1], b[2], b[3]);
        if (unit_of(ic) >= nunits) break;
        step(b[2], b[3], b[0], b[1]);
    }
    stamp(3);

    // slow region: chunks after the last whole round, plus the short tail chunk
    const uint64_t nfull = a.len / BPC;
    const uint64_t first_slow = nunits * kChunksPerUnit;
    const uint64_t nslow = nfull - first_slow + (a.len % BPC ? 1 : 0);
    const uint64_t gtid = uint64_t(blockIdx.x) * kBlockThreads + threadIdx.x;
    const bool crc_al4 = (reinterpret_cast<uintptr_t>(VERIFY ? a.crc_be : a.out_be) & 3u) == 0;
    if (gtid < nslow) {
        const uint64_t chunk = first_slow + gtid;
        const uint32_t sz = chunk < nfull ? uint32_t(BPC) : uint32_t(a.len % BPC);
        const uint32_t c = ~crc_run_lines(tb, 0xFFFFFFFFu, a.data + chunk * BPC, sz);
        if constexpr (VERIFY) {
            if ((sz == uint32_t(BPC) || a.check_short_tail) && load_be32(a.crc_be + 4 * chunk, crc_al4) != c)
                atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
        } else {
            store_be32(a.out_be + 4 * chunk, c, crc_al4);
        }
    }
}

// ---- segmented wave kernel: independent segments (blocks of a batch, packets) ----
//
// The wave kernel's rounds, over the union of every segment's whole 4 KiB rounds: global
// unit u (round-robin over waves as before) belongs to the segment with the largest
// unit_begin <= u — u / uniform when the host found equal-sized segments, else a scalar
// binary search over the descriptor array (wave-uniform, so SALU + scalar loads). Each
// round's segment view is resolved when the round is prefetched and travels with its
// buffer. Leftover chunks and short tails of every segment go to a per-segment slow pass.
constexpr uint32_t kInlineSegments = 16;  // small lists travel in the kernel arguments

struct SegLaunch {
    const DevSegment *seg;  // device array, or nullptr: use inl[] (nseg <= kInlineSegments)
    uint32_t nseg;
    uint64_t units;
    uint64_t uniform;
    unsigned long long *result;
    int check_short_tail;
    // stride != 0: packet i is {inl[0].data + i*stride, inl[0].crc + i*stride, inl[0].len,
    // key i << 32}, the last one with inl[1].len (uniform view only). Packets laid out at a
    // constant pitch in one arena need no descriptor array at all.
    uint64_t stride;
    DevSegment inl[kInlineSegments];
};

struct RoundView {
    const uint8_t *p;    // round data (or the table image past the wave's last round)
    uint8_t *crc;        // segment's CRC array
    uint64_t chunk0;     // segment chunk index of the round's first chunk
    uint64_t key0;       // key_base + chunk0
};

// UNI: every segment but the last has L.uniform units -> the segment is a 32-bit divide;
// otherwise a binary search. They are separate instantiations on purpose: a search loop in
// the hot loop's CFG (even untaken) makes the waitcnt pass drain the prefetch each step.
// ONE (A/B variant 49): a single segment, its view fixed at kernel start (no refresh branch).
// HOLD (compute at bpc 512): the wave kernel's held stores (kOptHoldStore). Each lane keeps
// the word it collects per 8 rounds together with its target address (rounds of one wave
// may belong to different segments), up to 8 octets, and stores them in bursts.
// (A fixed-depth unrolled search in place of the binary-search loop was 47 % slower on
// ragged batches: profiles/r01_kernel_study/seg_search_ab.jsonl, former variant 51.)
template <int BPC, bool VERIFY, bool UNI, bool ONE = false, bool HOLD = false>
__global__ __launch_bounds__(kBlockThreads) void crc32c_seg_kernel(SegLaunch L, const uint32_t *__restrict__ g_tab,
                                                                   const uint32_t *__restrict__ g_nib) {
    static_assert(BPC <= kRoundBytes && BPC % 64 == 0, "one-round units");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytesWave / 4];
    constexpr int G = BPC / 64;
    constexpr int kChunksPerUnit = kRoundBytes / BPC;

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane % G;
    const uint32_t lane_off = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint64_t nwaves = uint64_t(gridDim.x) * kWavesPerBlock;
    const uint64_t wave = uint64_t(blockIdx.x) * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t K = wave < L.units ? (L.units - wave + nwaves - 1) / nwaves : 0;

    // kernel-argument (inline) descriptors when the host passed no device array
    auto segp = [&](uint32_t i) -> const DevSegment * { return L.seg ? L.seg + i : L.inl + i; };
    static_assert(sizeof(DevSegment) == 40, "descriptor layout");
    auto seg_of = [&](uint64_t u) -> uint32_t {
        if constexpr (UNI) {  // unit counts stay < 2^32 (16 TiB per launch): 32-bit divide
            const uint32_t s = uint32_t(u) / uint32_t(L.uniform);
            return s < L.nseg ? s : L.nseg - 1;
        } else {
            uint32_t lo = 0, hi = L.nseg - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                const uint64_t ub = rfl64(segp(mid)->unit_begin);
                if (ub <= u) lo = mid;
                else hi = mid - 1;
            }
            return lo;
        }
    };
    // The prefetch stream's current segment, cached in scalar registers: a round inside it
    // needs only arithmetic; crossing into another segment costs one lookup (32-bit divide
    // or binary search) and the descriptor's scalar loads. Keeping those loads off the
    // common path matters: SMEM shares lgkmcnt with the LDS lookups and returns out of
    // order, so any in flight turns the pipelined lookup waits into lgkmcnt(0).
    uint64_t c_begin = 1, c_end = 0, c_key = 0;
    const uint8_t *c_data = nullptr;
    uint8_t *c_crc = nullptr;
    auto view = [&](uint64_t k) -> RoundView {
        RoundView v;
        if constexpr (ONE) {  // diagnostic: the wave kernel's round_ptr arithmetic, branch-free
            const uint64_t u = wave + k * nwaves;
            const bool in = k < K;
            v.p = in ? c_data + u * kRoundBytes : reinterpret_cast<const uint8_t *>(g_tab);
            v.crc = in ? c_crc : const_cast<uint8_t *>(reinterpret_cast<const uint8_t *>(g_tab));
            v.chunk0 = in ? u * kChunksPerUnit : 0;
            v.key0 = v.chunk0;
            return v;
        }
        if (k < K) {
            const uint64_t u = wave + k * nwaves;
            if (!ONE && (u < c_begin || u >= c_end)) {
                // descriptor fields come back in VGPRs (vector loads); made uniform here,
                // every per-round view computation below is SALU
                if (L.stride) {  // kernel-argument arithmetic only: no descriptor loads
                    const uint32_t si = seg_of(u);
                    c_begin = uint64_t(si) * L.uniform;
                    c_end = c_begin + (si + 1 < L.nseg ? L.uniform : L.inl[1].len / kRoundBytes);
                    c_data = L.inl[0].data + uint64_t(si) * L.stride;
                    c_crc = L.inl[0].crc + uint64_t(si) * L.stride;
                    c_key = uint64_t(si) << 32;
                } else {
                const DevSegment *sd = segp(seg_of(u));
                c_begin = rfl64(sd->unit_begin);
                c_end = c_begin + rfl64(sd->len) / kRoundBytes;
                c_data = reinterpret_cast<const uint8_t *>(rfl64(reinterpret_cast<uint64_t>(sd->data)));
                c_crc = reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(sd->crc)));
                c_key = rfl64(sd->key_base);
                }
            }
            const uint64_t r = u - c_begin;
            v.p = c_data + r * kRoundBytes;
            v.crc = c_crc;
            v.chunk0 = r * kChunksPerUnit;
            v.key0 = c_key + v.chunk0;
        } else {  // past the wave's last round: loads stay unconditional and read the
                  // cache-resident table image (see crc32c_wave_kernel); results are ignored
            v.p = reinterpret_cast<const uint8_t *>(g_tab);
            v.crc = const_cast<uint8_t *>(reinterpret_cast<const uint8_t *>(g_tab));
            v.chunk0 = 0;
            v.key0 = 0;
        }
        return v;
    };

    if constexpr (ONE) {
        const DevSegment *sd = segp(0);
        c_begin = rfl64(sd->unit_begin);
        c_end = c_begin + rfl64(sd->len) / kRoundBytes;
        c_data = reinterpret_cast<const uint8_t *>(rfl64(reinterpret_cast<uint64_t>(sd->data)));
        c_crc = reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(sd->crc)));
        c_key = rfl64(sd->key_base);
    }
    // lean fill (as the production wave kernel): one slice-table word per thread, replicated
    // in LDS; for G <= 32 the half-size fold image
    constexpr bool kHalfFold = G <= 32;
    const uint32_t tw = g_tab[threadIdx.x];
    u32x4 n0, n1;
    if constexpr (kHalfFold) {
        const uint32_t t = threadIdx.x;
        const uint32_t fk = 2 * (t >> 8) + ((t >> 3) & 1), fe = (t >> 4) & 15, fc = 4 * (t & 7);
        n0 = *reinterpret_cast<const u32x4 *>(g_nib + (fk * 16 + fe) * 64 + fc);
    } else {
        n0 = *reinterpret_cast<const u32x4 *>(g_nib + 8 * threadIdx.x);
        n1 = *reinterpret_cast<const u32x4 *>(g_nib + 8 * threadIdx.x + 4);
    }
    // views: cv* = rounds being consumed, pv* = rounds being prefetched by this step
    RoundView cv0 = view(0), cv1 = view(1);
    __builtin_amdgcn_sched_barrier(0);
    Round b[4];
    load_round_buf<true>(b[0], cv0.p, lane_off);
    load_round_buf<true>(b[1], cv1.p, lane_off);
    __builtin_amdgcn_sched_barrier(0);
    {
        const uint32_t tt = threadIdx.x, slice = tt >> 8, entry = tt & 255;
        u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
        const uint32_t slot0 = ((slice >> 1) << 16 | entry << 8 | (slice & 1) << 7) / 16;
#pragma unroll
        for (int r = 0; r < 8; ++r) l4[slot0 + ((r + tt) & 7)] = u32x4{tw, tw, tw, tw};
        if constexpr (kHalfFold) {
            reinterpret_cast<u32x4 *>(lds + kPoolFoldOff / 4)[tt] = n0;
        } else {
            u32x4 *dst = reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(lds) + kFoldLdsOff) + 2 * tt;
            dst[0] = n0;
            dst[1] = n1;
        }
    }
    lds_barrier();
    const Lut t(lds);
    const NibFold nf(lds);
    auto fold = [&](uint32_t x) -> uint32_t {
        if constexpr (kHalfFold) return fold_half(reinterpret_cast<const uint8_t *>(lds), x);
        return nf.apply(x);
    };
    const uint32_t init = j == 0 ? 0xFFFFFFFFu : 0u;
    RoundView pv0 = view(2), pv1 = view(3);

    // Descriptor pointers carry no address space, so plain dereferences would compile to
    // FLAT instructions, which count on lgkmcnt as well as vmcnt: every pipelined LDS wait
    // would become lgkmcnt(0) and the prefetch would drain. Casting to the global address
    // space keeps them global_load/store/atomic. Unconditional word loads (see the wave kernel).
    typedef __attribute__((address_space(1))) const uint32_t gcu32;
    typedef __attribute__((address_space(1))) uint32_t gu32;
    typedef __attribute__((address_space(1))) unsigned long long gu64;
    auto want_of = [&](const RoundView &v) -> uint32_t {
        if constexpr (VERIFY) return *(gcu32 *)(v.crc + 4 * (v.chunk0 + lane / G));
        return 0;
    };
    constexpr bool kHold = HOLD && !VERIFY && G == 8;
    uint32_t line = 0;                 // kHold: lane 8r + c collects chunk c of the octet's round r
    gu32 *laddr = nullptr;             //        and that word's destination (null: none this octet)
    uint32_t hold[kHold ? 8 : 1];      // hold[i] = the octet closed i octets ago
    gu32 *hold_addr[kHold ? 8 : 1];
    uint32_t nheld = 0;
    auto flush = [&]() {
#pragma unroll
        for (int i = 0; i < (kHold ? 8 : 0); ++i)
            if (uint32_t(i) < nheld && hold_addr[i]) *hold_addr[i] = __builtin_bswap32(~hold[i]);
        nheld = 0;
    };
    auto finish = [&](uint64_t k, const RoundView &v, uint32_t y, uint32_t want) {
        if constexpr (kHold) {
            if (k >= K) return;
            const uint32_t r = uint32_t(k & 7);
            // group c's lanes all hold chunk c's state (group_xor is a butterfly)
            const uint32_t got = uint32_t(__builtin_amdgcn_ds_bpermute(int(32 * (lane & 7)), int(y)));
            const bool mine = (lane >> 3) == r;
            line = mine ? got : line;
            laddr = mine ? (gu32 *)(v.crc + 4 * (v.chunk0 + (lane & 7))) : laddr;
            if (r == 7 || k + 1 == K) {
#pragma unroll
                for (int i = (kHold ? 7 : 0); i > 0; --i) {
                    hold[i] = hold[i - 1];
                    hold_addr[i] = hold_addr[i - 1];
                }
                hold[0] = line;
                hold_addr[0] = laddr;
                laddr = nullptr;
                if (++nheld == 8) flush();
            }
            return;
        }
        if (k >= K || j != 0) return;
        const uint32_t c = ~y;
        if constexpr (VERIFY) {
            if (__builtin_bswap32(want) != c)
                __hip_atomic_fetch_max((gu64 *)L.result, ~(unsigned long long)(v.key0 + lane / G),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            *(gu32 *)(v.crc + 4 * (v.chunk0 + lane / G)) = __builtin_bswap32(c);
        }
    };
    auto word = [](const Round &r, int i) -> uint32_t { return r.w[i >> 2][i & 3]; };

    // step: consume rounds k, k+1 (c0, c1; views cv0, cv1), prefetch k+2, k+3 (pv0, pv1).
    // Straight-line from the stored-word loads through the prefetch: the next step's views
    // (which branch) are resolved at the END of the step, after finish, so no branch sits
    // between this step's loads (LLVM would otherwise sink the word loads past the
    // prefetch and the waitcnt pass would drain it).
    auto step = [&](Round &c0, Round &c1, Round &p0, Round &p1, uint64_t k) {
        const uint32_t w0 = want_of(cv0), w1 = want_of(cv1);
        load_round_buf<true>(p0, pv0.p, lane_off);
        load_round_buf<true>(p1, pv1.p, lane_off);
        __builtin_amdgcn_sched_barrier(0);
        regroup(c0);
        regroup(c1);
        uint32_t x0 = init ^ word(c0, 0), x1 = init ^ word(c1, 0);
        Look l0 = lookups(t, x0), l1;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            l1 = lookups(t, x1);
            __builtin_amdgcn_sched_barrier(0);
            x0 = combine(l0, i < 15 ? word(c0, i < 15 ? i + 1 : 15) : 0u);
            __builtin_amdgcn_sched_barrier(0);
            if (i < 15) l0 = lookups(t, x0);
            __builtin_amdgcn_sched_barrier(0);
            x1 = combine(l1, i < 15 ? word(c1, i < 15 ? i + 1 : 15) : 0u);
            __builtin_amdgcn_sched_barrier(0);
        }
        finish(k, cv0, group_xor<G>(fold(x0)), w0);
        finish(k + 1, cv1, group_xor<G>(fold(x1)), w1);
        __builtin_amdgcn_sched_barrier(0);
        cv0 = pv0;
        cv1 = pv1;
        pv0 = view(k + 4);
        pv1 = view(k + 5);
    };
    for (uint64_t k = 0; k < K; k += 4) {
        step(b[0], b[1], b[2], b[3], k);
        if (k + 2 >= K) break;
        step(b[2], b[3], b[0], b[1], k + 2);
    }
    if constexpr (kHold) flush();

    // slow pass: per segment, the chunks after its last whole round and its short tail
    // (at most kChunksPerUnit of them). One chunk per thread, item i = segment
    // i / kChunksPerUnit, spread over the workgroups (item i -> block i % grid): a
    // segment's leftovers no longer run one after another on one lane, which made every
    // ragged batch wait for up to 7 serial chunks (~30 us at 1 GiB, tools/seg_search_ab.py).
    const uint64_t items = uint64_t(L.nseg) * kChunksPerUnit;
    for (uint64_t it = uint64_t(threadIdx.x) * gridDim.x + blockIdx.x; it < items;
         it += uint64_t(gridDim.x) * kBlockThreads) {
        const uint32_t si = uint32_t(it / kChunksPerUnit);
        DevSegment sd;
        if (L.stride) {
            sd = L.inl[0];
            sd.data += uint64_t(si) * L.stride;
            sd.crc += uint64_t(si) * L.stride;
            sd.len = si + 1 < L.nseg ? L.inl[0].len : L.inl[1].len;
            sd.key_base = uint64_t(si) << 32;
        } else {
            sd = *segp(si);
        }
        const uint64_t nfull = sd.len / BPC;
        const uint64_t first = (sd.len / kRoundBytes) * kChunksPerUnit;
        const uint64_t last = nfull + (sd.len % BPC ? 1 : 0);
        const uint64_t c = first + it % kChunksPerUnit;
        if (c < last) {
            const uint32_t sz = c < nfull ? uint32_t(BPC) : uint32_t(sd.len % BPC);
            const uint32_t v = ~crc_run_lines(t, 0xFFFFFFFFu, sd.data + c * BPC, sz);
            if constexpr (VERIFY) {
                if ((sz == uint32_t(BPC) || L.check_short_tail) && load_be32(sd.crc + 4 * c, true) != v)
                    atomicMax(L.result, ~(unsigned long long)(sd.key_base + c));
            } else {
                store_be32(sd.crc + 4 * c, v, true);
            }
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

// Diagnostic kernels for the per-launch fixed cost (variants 10-12): same grid and
// block as the production kernel; 10 = no LDS, 11 = 160 KiB LDS allocated but not
// written, 12 = LDS fill (tables + nibble image) + barrier.
template <int MODE>
__global__ __launch_bounds__(kBlockThreads) void fixed_cost_kernel(const uint32_t *__restrict__ g_tab,
                                                                   const uint32_t *__restrict__ g_nib,
                                                                   uint32_t *sink) {
    if constexpr (MODE == 10) {
        if (threadIdx.x == 1u << 30) sink[0] = 1;
    } else {
        __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytesWave / 4];
        if constexpr (MODE == 12) {
            uint32_t tv[kFillPerThread];
            fetch_tables(tv, g_tab);
            const u32x4 n0 = *reinterpret_cast<const u32x4 *>(g_nib + 8 * threadIdx.x);
            const u32x4 n1 = *reinterpret_cast<const u32x4 *>(g_nib + 8 * threadIdx.x + 4);
            store_tables(lds, tv);
            u32x4 *dst = reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(lds) + kFoldLdsOff) + 2 * threadIdx.x;
            dst[0] = n0;
            dst[1] = n1;
        }
        lds_barrier();
        if (lds[threadIdx.x] == 0x9E3779B9u && threadIdx.x == 1u << 30) sink[0] = 1;
    }
}

// ---- measurement-only kernels ------------------------------------------------

// Coalesced streaming read (1 KiB per wave-instruction): the achievable HBM read
// ceiling the CRC kernel is compared with.
template <bool NT>
__global__ __launch_bounds__(256) void stream_read_kernel(const uint8_t *__restrict__ d,
                                                          uint64_t n16, uint32_t *sink) {
    auto ld = [](const uint8_t *p) -> u32x4 {
        if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
        return ld16(p);
    };
    uint32_t acc = 0;
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const u32x4 a = ld(d + 16 * i), b = ld(d + 16 * (i + stride));
        const u32x4 c = ld(d + 16 * (i + 2 * stride)), e = ld(d + 16 * (i + 3 * stride));
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ e.x ^ e.y ^
               e.z ^ e.w;
    }
    for (; i < n16; i += stride) {
        const u32x4 a = ld(d + 16 * i);
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // keep the loads live
}

// Access-pattern probes (xor instead of table arithmetic), selected by `variant`:
//  0: chunk per lane, 8 x 16 B per 128 B line, nt loads   (the v1 CRC kernel's pattern)
//  1: same, default cache policy
//  2: G=8 lanes per chunk, one full 128 B line per chunk per instruction (coalesced)
//  3: G=4 lanes per chunk, 64 B per chunk per instruction
//  4: chunk per lane, 2 x 16 B (32 B) per lane per instruction pair, lines split over 4 lanes
template <int BPC, int VARIANT>
__global__ __launch_bounds__(kBlockThreads) void lane_read_kernel(const uint8_t *__restrict__ d,
                                                                  uint64_t nchunks, uint32_t *sink) {
    uint32_t acc = 0;
    const uint64_t tid = uint64_t(blockIdx.x) * kBlockThreads + threadIdx.x;
    const uint64_t nthreads = uint64_t(gridDim.x) * kBlockThreads;
    if constexpr (VARIANT <= 1) {
        for (uint64_t chunk = tid; chunk < nchunks; chunk += nthreads) {
            const uint8_t *p = d + chunk * BPC;
#pragma unroll
            for (int l = 0; l < BPC / 128; ++l) {
                u32x4 v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const u32x4 *q = reinterpret_cast<const u32x4 *>(p + 128 * l + 16 * i);
                    v[i] = VARIANT == 0 ? __builtin_nontemporal_load(q) : *q;
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) acc = (acc ^ v[i].x ^ v[i].y ^ v[i].z ^ v[i].w) * 3u;
            }
        }
    } else if constexpr (VARIANT == 2 || VARIANT == 3) {
        constexpr int G = VARIANT == 2 ? 8 : 4;
        const uint64_t groups = nthreads / G;
        for (uint64_t chunk = tid / G; chunk < nchunks; chunk += groups) {
            const uint8_t *p = d + chunk * BPC + 16 * (tid % G);
            constexpr int N = BPC / (16 * G), U = N < 8 ? N : 8;
#pragma unroll
            for (int t0 = 0; t0 < N; t0 += U) {
                u32x4 v[U];
#pragma unroll
                for (int i = 0; i < U; ++i) v[i] = *reinterpret_cast<const u32x4 *>(p + 16 * G * (t0 + i));
#pragma unroll
                for (int i = 0; i < U; ++i) acc = (acc ^ v[i].x ^ v[i].y ^ v[i].z ^ v[i].w) * 3u;
            }
        }
    } else {
        for (uint64_t chunk = tid; chunk < nchunks; chunk += nthreads) {
            const uint8_t *p = d + chunk * BPC;
#pragma unroll
            for (int l = 0; l < BPC / 128; ++l) {
                u32x4 v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const u32x4 *>(p + 128 * l + 16 * ((i * 2) % 8 + (i / 4)));
#pragma unroll
                for (int i = 0; i < 8; ++i) acc = (acc ^ v[i].x ^ v[i].y ^ v[i].z ^ v[i].w) * 3u;
            }
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

template <int BPC, bool V, int DEPTH, bool FOLD4>
hipError_t launch_r3(const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                     hipStream_t s) {
    constexpr uint64_t kUnit = BPC <= kRoundBytes ? kRoundBytes : BPC;
    const uint64_t units = a.len / kUnit;
    const uint64_t need = (units + kWavesPerBlock - 1) / kWavesPerBlock;
    const int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
    hipLaunchKernelGGL((crc32c_rounds_kernel<BPC, V, DEPTH, FOLD4>), dim3(grid), dim3(kBlockThreads), 0, s,
                       a, tab, fold);
    return hipGetLastError();
}

template <int BPC, bool V, int PAIR, bool NT = false, bool BUF = true, bool TRACE = false, bool PRIO = false,
          bool ANY_ORDER = false, int OPT = 0>
hipError_t launch_wave(const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                       hipStream_t s) {
    if constexpr (BPC > kRoundBytes) {
        return launch_r3<BPC, V, 1, true>(a, tab, fold, grid_cap, s);
    } else {
        constexpr int G = BPC / 64;
        constexpr int set = G == 8 ? 0 : G == 16 ? 1 : G == 32 ? 2 : 3;
        const uint32_t *nib = fold + kFoldWords + set * kFoldNibbleWords;
        const uint64_t units = (OPT & kOptPitch) != 0 ? ((a.npk - 1) << a.upp_log2) + a.last_len / kRoundBytes
                                                      : a.len / kRoundBytes;
        ChunkLaunch la = a;
        if constexpr ((OPT & (kOptFastTail | kOptSoloHalf)) != 0) la.m32 = fold + kFoldM32Off;
        const uint64_t need = (units + PAIR * kWavesPerBlock - 1) / (PAIR * kWavesPerBlock);
        int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
        if (grid < 1) grid = 1;
        if (ANY_ORDER || a.overlap_previous)  // AQL packet without the barrier bit (variant 16, opt-in flag)
            hipExtLaunchKernelGGL((crc32c_wave_r2_kernel<BPC, V, PAIR, NT, BUF, TRACE, PRIO, OPT>), dim3(grid),
                                  dim3(kBlockThreads), 0, s, nullptr, nullptr, hipExtAnyOrderLaunch, la, tab, nib);
        else
            hipLaunchKernelGGL((crc32c_wave_r2_kernel<BPC, V, PAIR, NT, BUF, TRACE, PRIO, OPT>), dim3(grid),
                               dim3(kBlockThreads), 0, s, la, tab, nib);
        return hipGetLastError();
    }
}

template <int BPC, bool V, bool TRACE = false>
hipError_t launch_pool(const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap, hipStream_t s) {
    if constexpr (BPC > 2048) {
        return launch_wave<BPC, V, 2, true>(a, tab, fold, grid_cap, s);
    } else {
        constexpr int G = BPC / 64;
        constexpr int set = G == 8 ? 0 : G == 16 ? 1 : 2;
        const uint32_t *nib = fold + kFoldWords + set * kFoldNibbleWords;
        const uint64_t units = a.len / kRoundBytes;
        const uint64_t need = (units + 2 * kWavesPerBlock - 1) / (2 * kWavesPerBlock);
        const int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
        if (a.overlap_previous)
            hipExtLaunchKernelGGL((crc32c_pool_kernel<BPC, V, TRACE>), dim3(grid > 0 ? grid : 1), dim3(kBlockThreads), 0,
                                  s, nullptr, nullptr, hipExtAnyOrderLaunch, a, tab, nib);
        else
            hipLaunchKernelGGL((crc32c_pool_kernel<BPC, V, TRACE>), dim3(grid > 0 ? grid : 1), dim3(kBlockThreads), 0, s,
                               a, tab, nib);
        return hipGetLastError();
    }
}

}  // namespace
}  // namespace hdfs3crc
