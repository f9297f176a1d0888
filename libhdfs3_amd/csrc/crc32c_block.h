// Block kernel: the production CRC32C kernel for bytesPerChecksum 512 and 1024 (G = 8 or 16
// lanes per chunk) over one contiguous run of chunks — a block, a local-reader window, a
// host-API segment. Same rounds, regroup, slice-by-4 lookups, LDS nibble fold and two
// software-pipelined chains per lane as crc32c_wave_kernel (crc32c_device.h),
// with the launch head rebuilt so the data stream never waits for table fetches:
//
//  * no table loads at all: every thread computes its slice-table entry T_s[e] from the
//    polynomial (8(s+1) shift/xor steps, s = thread >> 8 is wave-uniform) and writes its 32
//    bank copies; the lane-fold matrices M_j (advance over (G-1-j)*64 bytes) arrive as
//    columns in the kernel arguments (scalar loads, in flight with the rest of the
//    arguments), are staged in LDS by 16 lanes per wave and expanded into the half-size
//    nibble image by every thread. Round-1 wave traces put the old fill (4 KiB table + 16 KiB
//    fold image fetched from L2/MALL behind the first 32 MiB of round loads) at 4.5 us after
//    wave entry, and the first prefetch could only issue after it;
//  * a 4-round prologue (16 KiB in flight per wave, 256 KiB per CU) instead of 2 rounds,
//    with each step refilling the two buffers it just consumed at its END: in steady state
//    that is the same 8-16 KiB per wave in flight as before, but the head no longer drains.
//
// Kept bit-exact with the wave kernel: the parity tests run both.
#pragma once

#include "crc32c_device.h"

namespace hdfs3crc {
namespace {

constexpr int kColLdsOff = kPoolFoldOff + 16 * 1024;  // 144 KiB: staged fold columns (G x 32 words)
constexpr int kMaxColWords = 16 * 32;                  // G <= 16

struct BlockArgs {
    const uint8_t *data;
    uint64_t len;
    const uint8_t *crc_be;         // verify: stored BE32 words
    uint8_t *out_be;               // compute: BE32 words written here
    unsigned long long *result;    // verify: atomicMax(~first_bad) target
    uint64_t chunk_base;
    const uint32_t *dummy;         // >= 4 KiB, cache resident: target of prefetches past the last round
    uint32_t poly;                 // reflected polynomial (CRC32C 0x82F63B78 or CRC32 0xEDB88320)
    int check_short_tail;
    uint32_t cols[kMaxColWords];   // M_j by columns: word 32 j + b = M_j(1 << b), j < G
};

template <int BPC, bool VERIFY, bool HEAD4 = true>
__global__ __launch_bounds__(kBlockThreads) void crc32c_block_kernel(BlockArgs a) {
    static_assert(BPC == 512 || BPC == 1024, "G <= 16: fold columns in the kernel arguments");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytesWave / 4];
    constexpr int G = BPC / 64;
    constexpr int kChunksPerUnit = kRoundBytes / BPC;
    constexpr int kColsPerWave = G * 32 / kWavesPerBlock;  // 16 (G = 8) or 32 (G = 16)
    typedef __attribute__((address_space(1))) const uint32_t gcu32;
    typedef __attribute__((address_space(1))) uint32_t gu32;

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane % G;
    const uint32_t lane_off = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint32_t slot = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // Every argument the head needs, in ONE scalar round trip: left to itself the compiler
    // loads them in three dependent groups (behind the 64-bit divide and the K == 0 branch),
    // three kernel-argument latencies before the first data load.
    const uint8_t *data = a.data, *crc_be = a.crc_be;
    const uint8_t *dummy = reinterpret_cast<const uint8_t *>(a.dummy);
    const uint64_t len = a.len;
    const uint32_t poly = a.poly;
    uint32_t cv[kColsPerWave];
#pragma unroll
    for (int i = 0; i < kColsPerWave; ++i) cv[i] = a.cols[slot * kColsPerWave + i];
    asm volatile("" ::"s"(data), "s"(crc_be), "s"(dummy), "s"(len), "s"(poly));
    // unit (4 KiB round) counts stay below 2^32 (the host routes larger calls elsewhere), so
    // the per-wave round count K and every round index are 32-bit scalars: 64-bit compares
    // would go to the VALU and turn the end-of-stream selects into branches
    const uint32_t nunits = uint32_t(len / kRoundBytes);
    const uint32_t nwaves = gridDim.x * kWavesPerBlock;
    const uint32_t wave = blockIdx.x * kWavesPerBlock + slot;
    const uint32_t K = wave < nunits ? __builtin_amdgcn_readfirstlane((nunits - wave + nwaves - 1) / nwaves) : 0u;
    // round k of this wave is unit wave + k * nwaves; past the end, loads stay unconditional
    // (a branch around them makes the waitcnt pass drain at the loop head) and read `dummy`
    auto round_ptr = [&](uint32_t k) -> const uint8_t * {
        return k < K ? data + uint64_t(wave + k * nwaves) * kRoundBytes : dummy;
    };
    auto want_of = [&](uint32_t k) -> uint32_t {
        if constexpr (VERIFY) {
            const uint8_t *p = k < K ? crc_be + uint64_t(wave + k * nwaves) * (4 * kChunksPerUnit) : dummy;
            return *(gcu32 *)(p + 4 * (lane / G));
        }
        return 0;
    };

    // ---- head: the data stream first, then the tables (no global loads) -------------------
    Round b[4];
    uint32_t w[4];
    w[0] = want_of(0);
    w[1] = want_of(1);
    load_round_buf<true>(b[0], round_ptr(0), lane_off);
    load_round_buf<true>(b[1], round_ptr(1), lane_off);
    if constexpr (HEAD4) {
        w[2] = want_of(2);
        w[3] = want_of(3);
        load_round_buf<true>(b[2], round_ptr(2), lane_off);
        load_round_buf<true>(b[3], round_ptr(3), lane_off);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
        // slice table: T_s[e] = CRC of byte e followed by s zero bytes (crc32c_tables.h)
        const uint32_t t = threadIdx.x, s = t >> 8, e = t & 255;
        uint32_t c = e;
        const uint32_t steps = __builtin_amdgcn_readfirstlane(8 * (s + 1));
        for (uint32_t i = 0; i < steps; ++i) c = (c >> 1) ^ (poly & (0u - (c & 1u)));
        // 32 bank copies as 8 x ds_write_b128, rotated by thread (the lean fill's layout)
        u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
        const uint32_t slot0 = ((s >> 1) << 16 | e << 8 | (s & 1) << 7) / 16;
#pragma unroll
        for (int r = 0; r < 8; ++r) l4[slot0 + ((r + t) & 7)] = u32x4{c, c, c, c};
        // fold columns: wave `slot` stages words [slot * n, slot * n + n) from the arguments
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < kColsPerWave; ++i) v = lane == uint32_t(i) ? cv[i] : v;
        if (lane < uint32_t(kColsPerWave)) lds[kColLdsOff / 4 + slot * kColsPerWave + lane] = v;
    }
    lds_barrier();
    {
        // half-size nibble image (crc32c_pool_kernel's layout): word 4t + i holds M_jj(e << 4k)
        // for lane 4 (t & 7) + i (jj = that lane mod G), k = 2 (t >> 8) + ((t >> 3) & 1), e = (t >> 4) & 15
        const uint32_t t = threadIdx.x;
        const uint32_t k = 2 * (t >> 8) + ((t >> 3) & 1), e = (t >> 4) & 15, fc = 4 * (t & 7);
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t jj = (fc + i) % G;
            const u32x4 c4 = *reinterpret_cast<const u32x4 *>(lds + kColLdsOff / 4 + jj * 32 + 4 * k);
            o[i] = ((e & 1u) ? c4.x : 0u) ^ ((e & 2u) ? c4.y : 0u) ^ ((e & 4u) ? c4.z : 0u) ^ ((e & 8u) ? c4.w : 0u);
        }
        reinterpret_cast<u32x4 *>(lds + kPoolFoldOff / 4)[t] = u32x4{o[0], o[1], o[2], o[3]};
    }
    lds_barrier();
    const uint8_t *lds8 = reinterpret_cast<const uint8_t *>(lds);
    const Lut tab(lds);
    const uint32_t init = j == 0 ? 0xFFFFFFFFu : 0u;

    // ---- compute at bpc 512: held CRC-word stores (kOptHoldStore of the wave kernel) -------
    constexpr bool kHold = !VERIFY && G == 8;
    uint32_t line = 0;
    uint32_t hold[kHold ? 8 : 1];
    uint32_t nheld = 0;
    uint32_t hold_base = 0;
    auto flush = [&]() {
#pragma unroll
        for (int i = 0; i < (kHold ? 8 : 0); ++i) {
            if (uint32_t(i) < nheld) {
                const uint32_t k = 8 * (hold_base + nheld - 1 - i) + (lane >> 3);
                if (k < K)
                    *(gu32 *)(a.out_be + 4 * (uint64_t(wave + k * nwaves) * kChunksPerUnit + (lane & 7))) =
                        __builtin_bswap32(~hold[i]);
            }
        }
        hold_base += nheld;
        nheld = 0;
    };
    auto finish = [&](uint32_t k, uint32_t y, uint32_t want) {
        if constexpr (kHold) {
            if (k >= K) return;
            const uint32_t r = uint32_t(k & 7);
            const uint32_t got = uint32_t(__builtin_amdgcn_ds_bpermute(int(32 * (lane & 7)), int(y)));
            line = (lane >> 3) == r ? got : line;
            if (r == 7 || k + 1 == K) {
#pragma unroll
                for (int i = (kHold ? 7 : 0); i > 0; --i) hold[i] = hold[i - 1];
                hold[0] = line;
                if (++nheld == 8) flush();
            }
            return;
        }
        if (k >= K || j != 0) return;
        const uint64_t chunk = uint64_t(wave + k * nwaves) * kChunksPerUnit + lane / G;
        const uint32_t c = ~y;
        if constexpr (VERIFY) {
            if (__builtin_bswap32(want) != c) atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
        } else {
            *(gu32 *)(a.out_be + 4 * chunk) = __builtin_bswap32(c);
        }
    };
    auto word = [](const Round &r, int i) -> uint32_t { return r.w[i >> 2][i & 3]; };
    // two chains (rounds c0, c1), software-pipelined so one chain's lookups fly while the
    // other folds; then the lane fold and the chunk results
    auto rounds = [&](Round &c0, Round &c1, uint32_t k, uint32_t w0, uint32_t w1) {
        regroup(c0);
        regroup(c1);
        uint32_t x0 = init ^ word(c0, 0), x1 = init ^ word(c1, 0);
        Look l0 = lookups(tab, x0), l1;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            l1 = lookups(tab, x1);
            __builtin_amdgcn_sched_barrier(0);
            x0 = combine(l0, i < 15 ? word(c0, i < 15 ? i + 1 : 15) : 0u);
            __builtin_amdgcn_sched_barrier(0);
            if (i < 15) l0 = lookups(tab, x0);
            __builtin_amdgcn_sched_barrier(0);
            x1 = combine(l1, i < 15 ? word(c1, i < 15 ? i + 1 : 15) : 0u);
            __builtin_amdgcn_sched_barrier(0);
        }
        finish(k, group_xor<G>(fold_half(lds8, x0)), w0);
        finish(k + 1, group_xor<G>(fold_half(lds8, x1)), w1);
    };

    if constexpr (HEAD4) {
        // step k consumes rounds k, k+1 and, at its end, refills the same registers with k+4, k+5
        auto step = [&](Round &c0, Round &c1, uint32_t &w0, uint32_t &w1, uint32_t k) {
            rounds(c0, c1, k, w0, w1);
            __builtin_amdgcn_sched_barrier(0);
            w0 = want_of(k + 4);
            w1 = want_of(k + 5);
            load_round_buf<true>(c0, round_ptr(k + 4), lane_off);
            load_round_buf<true>(c1, round_ptr(k + 5), lane_off);
            __builtin_amdgcn_sched_barrier(0);
        };
        // No exit between the two steps of an iteration: a path that skips the second step
        // reaches the loop latch with only b[0], b[1] refilled, and the waitcnt pass merges
        // that path in and waits for every load at the loop head. The 0-3 leftover rounds
        // run after the loop.
        uint32_t k = 0;
        for (; k + 4 <= K; k += 4) {
            step(b[0], b[1], w[0], w[1], k);
            step(b[2], b[3], w[2], w[3], k + 2);
        }
        if (k < K) {
            step(b[0], b[1], w[0], w[1], k);
            if (k + 2 < K) step(b[2], b[3], w[2], w[3], k + 2);
        }
    } else {
        // the wave kernel's schedule: step k first prefetches k+2, k+3, then consumes k, k+1
        auto step = [&](Round &c0, Round &c1, Round &p0, Round &p1, uint32_t w0, uint32_t w1, uint32_t &pw0,
                        uint32_t &pw1, uint32_t k) {
            pw0 = want_of(k + 2);
            pw1 = want_of(k + 3);
            load_round_buf<true>(p0, round_ptr(k + 2), lane_off);
            load_round_buf<true>(p1, round_ptr(k + 3), lane_off);
            __builtin_amdgcn_sched_barrier(0);
            rounds(c0, c1, k, w0, w1);
        };
        for (uint32_t k = 0; k < K; k += 4) {
            step(b[0], b[1], b[2], b[3], w[0], w[1], w[2], w[3], k);
            if (k + 2 >= K) break;
            step(b[2], b[3], b[0], b[1], w[2], w[3], w[0], w[1], k + 2);
        }
    }
    if constexpr (kHold) flush();

    // slow region: chunks after the last whole round, plus the short tail chunk
    const uint64_t nfull = len / BPC;
    const uint64_t first_slow = uint64_t(nunits) * kChunksPerUnit;
    const uint64_t nslow = nfull - first_slow + (len % BPC ? 1 : 0);
    const uint64_t gtid = uint64_t(blockIdx.x) * kBlockThreads + threadIdx.x;
    const bool crc_al4 = (reinterpret_cast<uintptr_t>(VERIFY ? a.crc_be : a.out_be) & 3u) == 0;
    if (gtid < nslow) {
        const uint64_t chunk = first_slow + gtid;
        const uint32_t sz = chunk < nfull ? uint32_t(BPC) : uint32_t(len % BPC);
        const uint32_t c = ~crc_run_lines(tab, 0xFFFFFFFFu, data + chunk * BPC, sz);
        if constexpr (VERIFY) {
            if ((sz == uint32_t(BPC) || a.check_short_tail) && load_be32(a.crc_be + 4 * chunk, crc_al4) != c)
                atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
        } else {
            store_be32(a.out_be + 4 * chunk, c, crc_al4);
        }
    }
}

// cols: G x 32 fold columns of the ctx's polynomial (crc32c_tables.h build_fold_matrices,
// set G); dummy: a cache-resident buffer of at least 4 KiB
template <int BPC, bool V, bool HEAD4 = true>
hipError_t launch_block(const ChunkLaunch &c, uint32_t poly, const uint32_t *cols, const uint32_t *dummy,
                        int grid_cap, hipStream_t s) {
    constexpr int G = BPC / 64;
    BlockArgs a;
    a.data = c.data;
    a.len = c.len;
    a.crc_be = c.crc_be;
    a.out_be = c.out_be;
    a.result = c.result;
    a.chunk_base = c.chunk_base;
    a.dummy = dummy;
    a.poly = poly;
    a.check_short_tail = c.check_short_tail;
    for (int i = 0; i < G * 32; ++i) a.cols[i] = cols[i];
    for (int i = G * 32; i < kMaxColWords; ++i) a.cols[i] = 0;
    const uint64_t units = c.len / kRoundBytes;
    const uint64_t need = (units + 2 * kWavesPerBlock - 1) / (2 * kWavesPerBlock);
    uint64_t g = need < uint64_t(grid_cap) ? need : uint64_t(grid_cap);
    const int grid = int(g > 0 ? g : 1);
    if (c.overlap_previous)  // AQL packet without the barrier bit (HDFS3_LAUNCH_OVERLAP_PREVIOUS)
        hipExtLaunchKernelGGL((crc32c_block_kernel<BPC, V, HEAD4>), dim3(grid), dim3(kBlockThreads), 0, s, nullptr,
                              nullptr, hipExtAnyOrderLaunch, a);
    else
        hipLaunchKernelGGL((crc32c_block_kernel<BPC, V, HEAD4>), dim3(grid), dim3(kBlockThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace
}  // namespace hdfs3crc
