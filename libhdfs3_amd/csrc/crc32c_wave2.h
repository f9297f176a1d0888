// Two-workgroups-per-CU variant of the wave kernel (measurement library only, A/B variant 74;
// DESIGN.md §5.0).
//
// The production wave kernel fills all 160 KiB of a CU's LDS (32-way replicated slice-by-4
// tables + the half fold image), so a CU holds ONE workgroup, and with back-to-back launches
// the next launch's workgroup can only start on a CU after the previous one fully drained:
// every CU spends each launch's head (dispatch, table fill, first-data latency) pulling no HBM
// bytes, and a CU cannot borrow bandwidth from the others (the work-skew study, variant 73).
// Here the tables are slice-by-2 (T1, T0: 64 KiB replicated 32x) and the half fold image
// (16 KiB), 80 KiB per 512-thread workgroup: two workgroups per CU, so one launch's head
// overlaps the other workgroup's streaming. Same rounds, regroup, lane fold and keys as the
// wave kernel; one lookup per byte as before, but each 32-bit word is two dependent 16-bit
// steps: x -> T1[x.b0] ^ T0[x.b1] ^ (x >> 16) -> twice.
#pragma once

#include "crc32c_device.h"

namespace hdfs3crc {
namespace {

constexpr int kW2Threads = 512;
constexpr int kW2Waves = kW2Threads / 64;
constexpr int kW2TabBytes = 64 * 1024;                  // 2 slices x 256 entries x 32 copies x 4 B
constexpr int kW2FoldOff = kW2TabBytes;                 // half fold image, 16 KiB
constexpr int kW2LdsBytes = kW2TabBytes + 16 * 1024;    // 80 KiB

// entry e of slice s, copy c: byte e*256 + s*128 + 4c; lane l reads copy l % 32
struct Lut2 {
    const uint8_t *lds;
    uint32_t base[2];
    __device__ __forceinline__ explicit Lut2(const uint32_t *l) : lds(reinterpret_cast<const uint8_t *>(l)) {
        const uint32_t lane4 = (threadIdx.x & 31) * 4;
        base[0] = lane4;
        base[1] = lane4 | 0x80u;
    }
    // slice s at byte K of x: address {0, 0, x.byte K, base.byte0}
    template <int K>
    __device__ __forceinline__ uint32_t at(int s, uint32_t x) const {
        const uint32_t addr = __builtin_amdgcn_perm(x, base[s], 0x0C0C0000u | ((4u + K) << 8));
        return *reinterpret_cast<const uint32_t *>(lds + addr);
    }
};

struct Look2 {
    uint32_t v[2];
};
// the two lookups of a 16-bit step on state x (state ^ data already folded in)
__device__ __forceinline__ Look2 half_lookups(const Lut2 &t, uint32_t x) {
    Look2 l;
    l.v[0] = t.at<0>(1, x);  // T1[x.b0]
    l.v[1] = t.at<1>(0, x);  // T0[x.b1]
    return l;
}
__device__ __forceinline__ uint32_t half_combine(const Look2 &l, uint32_t x, uint32_t next) {
    return xor3(l.v[0], l.v[1], (x >> 16) ^ next);
}

template <int BPC, bool VERIFY>
// waves_per_eu(4): <= 128 VGPRs, so two 8-wave workgroups fit a CU's register file
__global__ __launch_bounds__(kW2Threads) __attribute__((amdgpu_waves_per_eu(4))) void crc32c_wave2_kernel(ChunkLaunch a, const uint32_t *__restrict__ g_tab,
                                                                   const uint32_t *__restrict__ g_nib) {
    static_assert(BPC <= 2048, "half fold image: G <= 32");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kW2LdsBytes / 4];
    constexpr int G = BPC / 64;
    constexpr int kChunksPerUnit = kRoundBytes / BPC;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane % G;
    const uint32_t lane_off = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint64_t nunits = a.len / kRoundBytes;
    const uint64_t nwaves = uint64_t(gridDim.x) * kW2Waves;
    const uint64_t wave = uint64_t(blockIdx.x) * kW2Waves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t K = wave < nunits ? (nunits - wave + nwaves - 1) / nwaves : 0;
    auto round_ptr = [&](uint64_t k) -> const uint8_t * {
        return k < K ? a.data + (wave + k * nwaves) * kRoundBytes : reinterpret_cast<const uint8_t *>(g_tab);
    };
    // table words first (thread t: slice t >> 8, entry t & 255), then the fold image (two
    // 16-byte pieces per thread), then the first two rounds, then the LDS fill
    const uint32_t t = threadIdx.x;
    const uint32_t tv = g_tab[t];
    u32x4 n[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t q = t + h * kW2Threads;
        const uint32_t fk = 2 * (q >> 8) + ((q >> 3) & 1), fe = (q >> 4) & 15, fc = 4 * (q & 7);
        n[h] = *reinterpret_cast<const u32x4 *>(g_nib + (fk * 16 + fe) * 64 + fc);
    }
    __builtin_amdgcn_sched_barrier(0);
    Round b[4];
    load_round_buf<true>(b[0], round_ptr(0), lane_off);
    load_round_buf<true>(b[1], round_ptr(1), lane_off);
    __builtin_amdgcn_sched_barrier(0);
    {
        u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
        const uint32_t slot0 = ((t & 255) << 8 | (t >> 8) << 7) / 16;
#pragma unroll
        for (int r = 0; r < 8; ++r) l4[slot0 + ((r + t) & 7)] = u32x4{tv, tv, tv, tv};
        u32x4 *f4 = reinterpret_cast<u32x4 *>(lds + kW2FoldOff / 4);
        f4[t] = n[0];
        f4[t + kW2Threads] = n[1];
    }
    lds_barrier();
    const Lut2 tb(lds);
    const uint32_t init = j == 0 ? 0xFFFFFFFFu : 0u;
    auto want_of = [&](uint64_t k) -> uint32_t {
        if constexpr (VERIFY) {
            const uint64_t kk = k < K ? k : K - 1;
            return *reinterpret_cast<const uint32_t *>(a.crc_be + 4 * ((wave + kk * nwaves) * kChunksPerUnit + lane / G));
        }
        return 0;
    };
    auto finish = [&](uint64_t k, uint32_t y, uint32_t want) {
        if (k >= K || j != 0) return;
        const uint64_t chunk = (wave + k * nwaves) * kChunksPerUnit + lane / G;
        const uint32_t c = ~y;
        if constexpr (VERIFY) {
            if (__builtin_bswap32(want) != c) atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
        } else {
            *reinterpret_cast<uint32_t *>(a.out_be + 4 * chunk) = __builtin_bswap32(c);
        }
    };
    auto word = [](const Round &r, int i) -> uint32_t { return r.w[i >> 2][i & 3]; };
    auto step = [&](Round &c0, Round &c1, Round &p0, Round &p1, uint64_t k) {
        const uint32_t w0 = want_of(k), w1 = want_of(k + 1);
        load_round_buf<true>(p0, round_ptr(k + 2), lane_off);
        load_round_buf<true>(p1, round_ptr(k + 3), lane_off);
        __builtin_amdgcn_sched_barrier(0);
        regroup(c0);
        regroup(c1);
        // 32 half-steps per round; the two chains alternate so each has its lookups in flight
        // while the other combines
        uint32_t x0 = init ^ word(c0, 0), x1 = init ^ word(c1, 0);
        Look2 l0 = half_lookups(tb, x0), l1;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < 32; ++h) {
            // next data word enters after the second half-step of each word
            const bool wend = (h & 1) != 0;
            const int wi = h >> 1;
            l1 = half_lookups(tb, x1);
            __builtin_amdgcn_sched_barrier(0);
            x0 = half_combine(l0, x0, wend && wi < 15 ? word(c0, wend && wi < 15 ? wi + 1 : 15) : 0u);
            __builtin_amdgcn_sched_barrier(0);
            if (h < 31) l0 = half_lookups(tb, x0);
            __builtin_amdgcn_sched_barrier(0);
            x1 = half_combine(l1, x1, wend && wi < 15 ? word(c1, wend && wi < 15 ? wi + 1 : 15) : 0u);
            __builtin_amdgcn_sched_barrier(0);
        }
        const uint8_t *l8 = reinterpret_cast<const uint8_t *>(lds);
        finish(k, group_xor<G>(fold_half<kW2FoldOff>(l8, x0)), w0);
        finish(k + 1, group_xor<G>(fold_half<kW2FoldOff>(l8, x1)), w1);
    };
    for (uint64_t k = 0; k < K; k += 4) {
        step(b[0], b[1], b[2], b[3], k);
        if (k + 2 >= K) break;
        step(b[2], b[3], b[0], b[1], k + 2);
    }
    // slow region: chunks after the last whole round, plus the short tail chunk (byte-table
    // path on T0)
    const uint64_t nfull = a.len / BPC;
    const uint64_t first_slow = nunits * kChunksPerUnit;
    const uint64_t nslow = nfull - first_slow + (a.len % BPC ? 1 : 0);
    const uint64_t gtid = uint64_t(blockIdx.x) * kW2Threads + threadIdx.x;
    if (gtid < nslow) {
        const uint64_t chunk = first_slow + gtid;
        const uint32_t sz = chunk < nfull ? uint32_t(BPC) : uint32_t(a.len % BPC);
        const uint8_t *p = a.data + chunk * BPC;
        uint32_t c = 0xFFFFFFFFu;
        for (uint32_t i = 0; i < sz; ++i) c = tb.at<0>(0, (c ^ p[i]) & 0xFFu) ^ (c >> 8);
        c = ~c;
        if constexpr (VERIFY) {
            if ((sz == uint32_t(BPC) || a.check_short_tail) && load_be32(a.crc_be + 4 * chunk, true) != c)
                atomicMax(a.result, ~(unsigned long long)(a.chunk_base + chunk));
        } else {
            store_be32(a.out_be + 4 * chunk, c, true);
        }
    }
}

template <int BPC, bool V>
hipError_t launch_wave2(const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap, hipStream_t s,
                        int wg_per_cu = 2) {
    if constexpr (BPC > 2048) {
        return hipErrorInvalidValue;
    } else {
        constexpr int G = BPC / 64;
        constexpr int set = G == 8 ? 0 : G == 16 ? 1 : 2;
        const uint32_t *nib = fold + kFoldWords + set * kFoldNibbleWords;
        const uint64_t units = a.len / kRoundBytes;
        const uint64_t need = (units + 2 * kW2Waves - 1) / (2 * kW2Waves);
        // 2: both LDS halves of every CU; 1: one workgroup per CU, so an overlapped next launch
        // finds the other half free and its head runs while this launch streams
        const uint64_t cap = uint64_t(wg_per_cu) * uint64_t(grid_cap);
        const int grid = int(need < cap ? need : cap) > 0 ? int(need < cap ? need : cap) : 1;
        if (a.overlap_previous)
            hipExtLaunchKernelGGL((crc32c_wave2_kernel<BPC, V>), dim3(grid), dim3(kW2Threads), 0, s, nullptr, nullptr,
                                  hipExtAnyOrderLaunch, a, tab, nib);
        else
            hipLaunchKernelGGL((crc32c_wave2_kernel<BPC, V>), dim3(grid), dim3(kW2Threads), 0, s, a, tab, nib);
        return hipGetLastError();
    }
}

}  // namespace
}  // namespace hdfs3crc
