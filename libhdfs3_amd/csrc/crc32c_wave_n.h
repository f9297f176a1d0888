// Lab-only (crc32c_experiments.hip, libhdfs3_crc_lab.so): the round kernel of crc32c_wave.h with
// NCH lookup chains per step instead of two, and the workgroup size as a parameter, for the
// geometry study of DESIGN.md §5.0.1 (round 3: a plain read of 128 MiB in rounds runs fastest with
// 4 waves per CU, but 4 waves of two chains each cannot hide the LDS lookup latency).
//
// A step consumes NCH rounds as NCH chains on a rotating schedule: chain c's lookups of word i+1
// go out right after its combine of word i, so NCH - 1 other (combine, lookups) groups separate
// every lookup from its use (NCH = 2 is exactly the production schedule). The next step's NCH
// rounds are requested once this step's rounds have landed (late prefetch, as production).
// Contiguous blocks only; the last step is interleaved (no solo step).
#pragma once

#include "crc32c_wave.h"

namespace hdfs3crc {
namespace {

template <int BPC, bool VERIFY, bool HOLD, int NCH, int TPB, class Walk>
__device__ __forceinline__ void wave_rounds_n(Walk &walk, uint32_t *lds, const uint32_t *__restrict__ g_tab,
                                              const uint32_t *__restrict__ g_nib, unsigned long long *result) {
    constexpr int G = BPC / 64;
    constexpr bool kHalfFold = G <= 32;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane % G;
    const uint32_t lane_off = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint32_t K = walk.K;

    constexpr int kFillIters = 1024 / TPB;
    static_assert(kFillIters * TPB == 1024, "TPB divides 1024");
    uint32_t tw[kFillIters];
    u32x4 n0[kFillIters], n1[kFillIters];
#pragma unroll
    for (int f = 0; f < kFillIters; ++f) {
        const uint32_t t = threadIdx.x + f * TPB;
        tw[f] = g_tab[t];
        if constexpr (kHalfFold) {
            const uint32_t fk = 2 * (t >> 8) + ((t >> 3) & 1), fe = (t >> 4) & 15, fc = 4 * (t & 7);
            n0[f] = *reinterpret_cast<const u32x4 *>(g_nib + (fk * 16 + fe) * 64 + fc);
        } else {
            n0[f] = *reinterpret_cast<const u32x4 *>(g_nib + 8 * t);
            n1[f] = *reinterpret_cast<const u32x4 *>(g_nib + 8 * t + 4);
        }
    }
    WView cv[NCH], pv[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) cv[i] = walk.view(i);
    __builtin_amdgcn_sched_barrier(0);
    Round A[NCH], B[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) load_round_buf<true>(A[i], cv[i].p, lane_off);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < kFillIters; ++f) {
        const uint32_t tt = threadIdx.x + f * TPB, slice = tt >> 8, entry = tt & 255;
        u32x4 *l4 = reinterpret_cast<u32x4 *>(lds);
        const uint32_t slot0 = ((slice >> 1) << 16 | entry << 8 | (slice & 1) << 7) / 16;
        const uint32_t w = tw[f];
#pragma unroll
        for (int r = 0; r < 8; ++r) l4[slot0 + ((r + tt) & 7)] = u32x4{w, w, w, w};
        if constexpr (kHalfFold) {
            reinterpret_cast<u32x4 *>(lds + kHalfFoldOff / 4)[tt] = n0[f];
        } else {
            u32x4 *dst = reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(lds) + kFoldLdsOff) + 2 * tt;
            dst[0] = n0[f];
            dst[1] = n1[f];
        }
    }
    lds_barrier();
    const Lut t(lds);
    const NibFold nf(lds);
    auto fold = [&](uint32_t x) -> uint32_t {
        if constexpr (kHalfFold) return fold_half(reinterpret_cast<const uint8_t *>(lds), x);
        return nf.apply(x);
    };
    const uint32_t woff = 4 * (lane / G);
#pragma unroll
    for (int i = 0; i < NCH; ++i) pv[i] = walk.view(NCH + i);

    auto wrsrc = [](const WView &v) {
        return __builtin_amdgcn_make_buffer_rsrc(v.w, 0, 4 * (kRoundBytes / BPC), 0x00020000);
    };
    auto want_of = [&](const WView &v) -> uint32_t {
        if constexpr (VERIFY) return __builtin_amdgcn_raw_buffer_load_b32(wrsrc(v), woff, 0, 0);
        return 0;
    };
    constexpr bool kHold = HOLD && !VERIFY && G == 8;
    uint32_t line = 0;
    uint32_t hold[kHold ? 8 : 1];
    uint32_t nheld = 0, hold_base = 0;
    auto flush = [&]() {
#pragma unroll
        for (int i = 0; i < (kHold ? 8 : 0); ++i) {
            if (uint32_t(i) < nheld) {
                const uint32_t kk = 8 * (hold_base + nheld - 1 - i) + (lane >> 3);
                if (kk < K) *(gu32 *)((gu8 *)walk.view(kk).w + 4 * (lane & 7)) = __builtin_bswap32(hold[i]);
            }
        }
        hold_base += nheld;
        nheld = 0;
    };
    auto finish = [&](uint32_t k, const WView &v, uint32_t y, uint32_t want) {
        if constexpr (kHold) {
            if (k >= K) return;
            const uint32_t r = k & 7;
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
        if constexpr (VERIFY) {
            if (__builtin_bswap32(want) != y)
                __hip_atomic_fetch_max((gu64 *)result, ~(unsigned long long)(v.key + lane / G), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bswap32(y), wrsrc(v), woff, 0, 0);
        }
    };
    auto word = [](const Round &r, int i) -> uint32_t { return r.w[i >> 2][i & 3]; };
    // NCH chains on the rotating schedule (file comment)
    auto chains = [&](Round (&c)[NCH], uint32_t (&x)[NCH]) {
        Look l[NCH];
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            x[ch] = word(c[ch], 0);
            l[ch] = lookups(t, x[ch]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {
                x[ch] = combine(l[ch], i < 15 ? word(c[ch], i < 15 ? i + 1 : 15) : 0u);
                if (i < 15) l[ch] = lookups(t, x[ch]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    auto step = [&](Round (&C)[NCH], Round (&P)[NCH], uint32_t k) {
        uint32_t w[NCH];
#pragma unroll
        for (int i = 0; i < NCH; ++i) w[i] = want_of(cv[i]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NCH; ++i) regroup(C[i]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NCH; ++i) load_round_buf<true>(P[i], pv[i].p, lane_off);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t x[NCH];
        chains(C, x);
#pragma unroll
        for (int i = 0; i < NCH; ++i) finish(k + i, cv[i], group_xor<G>(fold(x[i])), w[i]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            cv[i] = pv[i];
            pv[i] = walk.view(k + 2 * NCH + i);
        }
    };
    const uint32_t nr = (K + NCH - 1) / NCH * NCH;
    for (uint32_t k = 0; k < nr; k += 2 * NCH) {
        step(A, B, k);
        if (k + NCH >= nr) break;
        step(B, A, k + NCH);
    }
    if constexpr (kHold) flush();
}

template <int BPC, bool VERIFY, int NCH, int TPB>
__global__ __launch_bounds__(TPB) void crc32c_wave_n_kernel(ChunkLaunch a, const uint32_t *__restrict__ g_tab,
                                                            const uint32_t *__restrict__ g_nib) {
    static_assert(BPC <= kRoundBytes && BPC % 512 == 0, "one-round units");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytesWave / 4];
    constexpr int kCpu = kRoundBytes / BPC;
    constexpr int kWpb = TPB / 64;
    const uint64_t nwaves = uint64_t(gridDim.x) * kWpb;
    const uint64_t wave = uint64_t(blockIdx.x) * kWpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *words = VERIFY ? const_cast<uint8_t *>(a.crc_be) : a.out_be;
    const uint8_t *dummy = reinterpret_cast<const uint8_t *>(g_tab);
    const uint64_t nunits = a.len / kRoundBytes;
    BlockWalk<kCpu> w{a.data, words, a.chunk_base, wave, nwaves,
                      uint32_t(rfl64(wave < nunits ? (nunits - wave + nwaves - 1) / nwaves : 0)), dummy};
    wave_rounds_n<BPC, VERIFY, !VERIFY && BPC == 512, NCH, TPB>(w, lds, g_tab, g_nib, a.result);
    slow_region<BPC, VERIFY, TPB>(lds, a.data, words, a.len, a.chunk_base, a.check_short_tail, a.result);
}

template <int BPC, bool V, int NCH, int TPB>
hipError_t launch_wave_n(const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                         hipStream_t s) {
    constexpr int G = BPC / 64;
    constexpr int set = G == 8 ? 0 : G == 16 ? 1 : G == 32 ? 2 : 3;
    const uint32_t *nib = fold + kFoldAffineOff + set * kFoldNibbleWords;
    const uint64_t units = a.len / kRoundBytes;
    const uint64_t need = (units + NCH * (TPB / 64) - 1) / (NCH * (TPB / 64));
    int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
    if (grid < 1) grid = 1;
    if (a.overlap_previous)
        hipExtLaunchKernelGGL((crc32c_wave_n_kernel<BPC, V, NCH, TPB>), dim3(grid), dim3(TPB), 0, s, nullptr, nullptr,
                              hipExtAnyOrderLaunch, a, tab, nib);
    else
        hipLaunchKernelGGL((crc32c_wave_n_kernel<BPC, V, NCH, TPB>), dim3(grid), dim3(TPB), 0, s, a, tab, nib);
    return hipGetLastError();
}

}  // namespace
}  // namespace hdfs3crc
