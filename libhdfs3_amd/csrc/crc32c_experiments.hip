// Kernel variants kept for in-process A/B and diagnostics (hdfs3x_set_variant, tools/ab.py;
// DESIGN.md §5.0), and the read-ceiling kernels of the bench. Linked into the measurement
// library libhdfs3_crc_lab.so only (HDFS3_LAB=1); the product libhdfs3_crc.so never sees it.
// Bit-exact variants are parity-tested (tests/test_gpu_parity.py); the diagnostic ones
// (no HBM / no math / fake lookups / timestamps) give wrong results on purpose.
#include "crc32c_block.h"
#include "crc32c_wave2.h"
#include "crc32c_wave.h"

namespace hdfs3crc {
namespace {

template <int BPC, bool V>
hipError_t launch_exp(int variant, const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                      hipStream_t s) {
    switch (variant) {
    case 1: return launch_r3<BPC, V, 1, false>(a, tab, fold, grid_cap, s);   // first round kernel
    case 2: return launch_r3<BPC, V, 1, true>(a, tab, fold, grid_cap, s);    // + bitop3 fold
    case 3: return launch_r3<BPC, V, 2, true>(a, tab, fold, grid_cap, s);    // + 2-deep prefetch
    case 4: return launch_wave<BPC, V, 1>(a, tab, fold, grid_cap, s);        // nibble fold, 1 chain
    case 5: return launch_wave<BPC, V, 2, false>(a, tab, fold, grid_cap, s); // 2 chains, default-policy loads
    case 7: return launch_wave<BPC, V, 2, true, false>(a, tab, fold, grid_cap, s);  // nt via global_load
    case 9: {  // diagnostic: full grid, LDS fill + barrier, no rounds (per-launch fixed cost)
        ChunkLaunch e = a;
        e.len = 0;
        constexpr int G = BPC <= kRoundBytes ? BPC / 64 : 64;
        constexpr int set = G == 8 ? 0 : G == 16 ? 1 : G == 32 ? 2 : 3;
        if constexpr (BPC <= kRoundBytes)
            hipLaunchKernelGGL((crc32c_wave_r2_kernel<BPC, V, 1>), dim3(grid_cap), dim3(kBlockThreads), 0, s, e,
                               tab, fold + kFoldWords + set * kFoldNibbleWords);
        return hipGetLastError();
    }
    case 10:
        hipLaunchKernelGGL(fixed_cost_kernel<10>, dim3(grid_cap), dim3(kBlockThreads), 0, s, tab, fold, nullptr);
        return hipGetLastError();
    case 11:
        hipLaunchKernelGGL(fixed_cost_kernel<11>, dim3(grid_cap), dim3(kBlockThreads), 0, s, tab, fold, nullptr);
        return hipGetLastError();
    case 12:
        hipLaunchKernelGGL(fixed_cost_kernel<12>, dim3(grid_cap), dim3(kBlockThreads), 0, s, tab,
                           fold + kFoldWords, nullptr);
        return hipGetLastError();
    case 13: {  // diagnostic: production kernel + per-wave timestamps (tools/wave_trace.py)
        if (!g_trace) return hipErrorInvalidValue;
        ChunkLaunch e = a;
        e.trace = g_trace;
        return launch_wave<BPC, V, 2, true, true, true>(e, tab, fold, grid_cap, s);
    }
    case 14: return launch_wave<BPC, V, 2, true, true, false, true>(a, tab, fold, grid_cap, s);  // + s_setprio
    case 16: return launch_wave<BPC, V, 2, true, true, false, false, true>(a, tab, fold, grid_cap, s);
    case 15: {  // 14 with timestamps
        if (!g_trace) return hipErrorInvalidValue;
        ChunkLaunch e = a;
        e.trace = g_trace;
        return launch_wave<BPC, V, 2, true, true, true, true>(e, tab, fold, grid_cap, s);
    }
    case 18: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptFillFirst>(a, tab, fold, grid_cap, s);
    case 19: {  // 18 with timestamps
        if (!g_trace) return hipErrorInvalidValue;
        ChunkLaunch e = a;
        e.trace = g_trace;
        return launch_wave<BPC, V, 2, true, true, true, false, false, kOptFillFirst>(e, tab, fold, grid_cap, s);
    }
    case 20: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptFillWait>(a, tab, fold, grid_cap, s);
    case 21: {  // 20 with timestamps
        if (!g_trace) return hipErrorInvalidValue;
        ChunkLaunch e = a;
        e.trace = g_trace;
        return launch_wave<BPC, V, 2, true, true, true, false, false, kOptFillWait>(e, tab, fold, grid_cap, s);
    }
    case 22: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptNoHbm>(a, tab, fold, grid_cap, s);
    case 23: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptNoFill>(a, tab, fold, grid_cap, s);
    case 24: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptNoMath>(a, tab, fold, grid_cap, s);
    case 25:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptNoMath | kOptNoFill>(a, tab, fold, grid_cap, s);
    case 26: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptNibPerm | kOptWantBuf>(a, tab, fold, grid_cap, s);
    case 27: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptPf2 | kOptWantBuf>(a, tab, fold, grid_cap, s);
    case 28:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptPf2 | kOptNibPerm | kOptWantBuf>(a, tab, fold,
                                                                                                       grid_cap, s);
    case 29: {  // 28 with timestamps
        if (!g_trace) return hipErrorInvalidValue;
        ChunkLaunch e = a;
        e.trace = g_trace;
        return launch_wave<BPC, V, 2, true, true, true, false, false, kOptPf2 | kOptNibPerm | kOptWantBuf>(e, tab, fold,
                                                                                                      grid_cap, s);
    }
    case 30: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptWantBuf>(a, tab, fold, grid_cap, s);
    case 31:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptWantBuf | kOptLate>(a, tab, fold, grid_cap, s);
    case 32:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptWantBuf | kOptSplit>(a, tab, fold, grid_cap, s);
    case 33: return launch_wave<BPC, V, 2, true, true, false, true, false, kOptWantBuf | kOptLate>(a, tab, fold, grid_cap, s);
    case 35: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptFakeLut>(a, tab, fold, grid_cap, s);
    case 40: return launch_pool<BPC, V>(a, tab, fold, grid_cap, s);
    case 44: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill>(a, tab, fold, grid_cap, s);
    case 45:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptNoStore>(a, tab, fold,
                                                                                                    grid_cap, s);
    case 46:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptLineStore>(a, tab, fold,
                                                                                                      grid_cap, s);
    case 47:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptHoldStore>(a, tab, fold,
                                                                                                      grid_cap, s);
    case 48:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptNibPerm>(a, tab, fold, grid_cap,
                                                                                                    s);
    case 43: return launch_wave<BPC, V, 2, true, true, false, false, false, kOptNtStore>(a, tab, fold, grid_cap, s);
    case 42:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptVgprFold | kOptWantBuf>(a, tab, fold, grid_cap,
                                                                                                   s);
    case 41: {  // 40 with timestamps
        if (!g_trace) return hipErrorInvalidValue;
        ChunkLaunch e = a;
        e.trace = g_trace;
        return launch_pool<BPC, V, true>(e, tab, fold, grid_cap, s);
    }
    case 36:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptSlotRegion | kOptWantBuf>(a, tab, fold, grid_cap,
                                                                                                    s);
    case 37: {  // 36 with timestamps
        if (!g_trace) return hipErrorInvalidValue;
        ChunkLaunch e = a;
        e.trace = g_trace;
        return launch_wave<BPC, V, 2, true, true, true, false, false, kOptSlotRegion | kOptWantBuf>(e, tab, fold,
                                                                                                   grid_cap, s);
    }
    case 38:
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptSlotRegion | kOptWantBuf | kOptNoMath>(
            a, tab, fold, grid_cap, s);
    case 70:  // production + two steps loaded before the fill (kOptHead2)
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptHead2>(a, tab, fold, grid_cap, s);
    case 71:  // 70, overlapped launch
        return launch_wave<BPC, V, 2, true, true, false, false, true, kOptLeanFill | kOptHead2>(a, tab, fold, grid_cap, s);
    case 72:  // production + the fast tail (kOptFastTail)
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptFastTail>(a, tab, fold, grid_cap, s);
    case 73:  // production + uneven work per workgroup (kOptSkew)
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptSkew>(a, tab, fold, grid_cap, s);
    case 76:  // diagnostic: production with the last step's table CRC skipped (kOptDiagTail)
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptDiagTail>(a, tab, fold, grid_cap, s);
    case 78:  // production + the last two rounds as single chains, one after the other (kOptSoloTail)
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptSoloTail>(a, tab, fold, grid_cap, s);
    case 79:  // 78 with held compute stores (compute at 512: the production store path)
        return launch_wave<BPC, V, 2, true, true, false, false, false,
                           kOptLeanFill | kOptSoloTail | (!V && BPC == 512 ? kOptHoldStore : 0)>(a, tab, fold, grid_cap, s);
    case 80:  // diagnostic: 76, but the last step's lookups are issued without their chain
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptDiagTail | kOptDiagTailLut>(
            a, tab, fold, grid_cap, s);
    case 82:  // 78 + the very last round as two half chains joined in VALU (kOptSoloHalf)
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptSoloTail | kOptSoloHalf>(
            a, tab, fold, grid_cap, s);
    case 77:  // diagnostic: production with every step's table CRC skipped (lean-fill variant 24)
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill | kOptNoMath>(a, tab, fold, grid_cap, s);
    case 74:    // two 512-thread workgroups per CU, slice-by-2 tables (crc32c_wave2.h)
    case 75: {  // the same kernel, one workgroup per CU per launch (grid = CUs)
        if constexpr (BPC <= 2048) {
            return launch_wave2<BPC, V>(a, tab, fold, grid_cap, s, variant == 74 ? 2 : 1);
        } else {
            return launch_wave<BPC, V, 2, true, true, false, false, false, kOptLeanFill>(a, tab, fold, grid_cap, s);
        }
    }
    case 60:  // block kernel (crc32c_block.h): computed tables + 4-round head
    case 61: {  // block kernel with the wave kernel's 2-round head (tables still computed)
        if constexpr (BPC == 512 || BPC == 1024) {
            if (!a.fold_host || !a.poly) return hipErrorInvalidValue;
            const uint32_t *cols = a.fold_host + (BPC == 512 ? 0 : 8 * 32);
            return variant == 60 ? launch_block<BPC, V, true>(a, a.poly, cols, tab, grid_cap, s)
                                 : launch_block<BPC, V, false>(a, a.poly, cols, tab, grid_cap, s);
        } else {
            constexpr int kOpt = (BPC <= kRoundBytes ? kOptLeanFill : 0);
            return launch_wave<BPC, V, 2, true, true, false, false, false, kOpt>(a, tab, fold, grid_cap, s);
        }
    }
    case 90:
    case 91: {  // the round-2 production kernel (before crc32c_wave.h): solo tail when overlapped
        constexpr int kOpt = (BPC <= kRoundBytes ? kOptLeanFill : 0) | (!V && BPC == 512 ? kOptHoldStore : 0);
        if (a.overlap_previous) {
            if constexpr (V && BPC <= kRoundBytes) {
                if (a.len <= (uint64_t(256) << 20))
                    return launch_wave<BPC, V, 2, true, true, false, false, true, kOpt | kOptSoloTail>(a, tab, fold,
                                                                                                      grid_cap, s);
            }
            return launch_wave<BPC, V, 2, true, true, false, false, true, kOpt>(a, tab, fold, grid_cap, s);
        }
        return launch_wave<BPC, V, 2, true, true, false, false, false, kOpt>(a, tab, fold, grid_cap, s);
    }
    case 92:  // the round-3 kernel with its prefetch issued at the start of each step (early)
        if constexpr (BPC <= kRoundBytes) return launch_wave3<BPC, V, false, 0>(a, tab, fold, grid_cap, s);
        return hipErrorInvalidValue;
    case 93:  // the round-3 kernel, late prefetch, no solo last step
        if constexpr (BPC <= kRoundBytes) return launch_wave3<BPC, V, false, 1, false>(a, tab, fold, grid_cap, s);
        return hipErrorInvalidValue;
    case 94:  // 92 + solo last step when overlapped
        if constexpr (BPC <= kRoundBytes) return launch_wave3<BPC, V, false, 0, V>(a, tab, fold, grid_cap, s);
        return hipErrorInvalidValue;
    case 97:  // late prefetch in the first step of each pair, early in the second (+ solo)
        if constexpr (BPC <= kRoundBytes) return launch_wave3<BPC, V, false, 3, V>(a, tab, fold, grid_cap, s);
        return hipErrorInvalidValue;
    case 98:  // early in the first step of each pair, late in the second (+ solo)
        if constexpr (BPC <= kRoundBytes) return launch_wave3<BPC, V, false, 4, V>(a, tab, fold, grid_cap, s);
        return hipErrorInvalidValue;
    case 96:  // production with the prefetch held until every load of the wave landed (LATE 2)
        if constexpr (BPC <= kRoundBytes) return launch_wave3<BPC, V, false, 2, V>(a, tab, fold, grid_cap, s);
        return hipErrorInvalidValue;
    case 34: {  // 24 (no table math) with timestamps
        if (!g_trace) return hipErrorInvalidValue;
        ChunkLaunch e = a;
        e.trace = g_trace;
        return launch_wave<BPC, V, 2, true, true, true, false, false, kOptNoMath>(e, tab, fold, grid_cap, s);
    }
    default: return hipErrorInvalidValue;
    }
}

template <int BPC>
hipError_t launch_exp_v(int variant, const ChunkLaunch &a, bool verify, const uint32_t *tab, const uint32_t *fold,
                        int grid_cap, hipStream_t s) {
    return verify ? launch_exp<BPC, true>(variant, a, tab, fold, grid_cap, s)
                  : launch_exp<BPC, false>(variant, a, tab, fold, grid_cap, s);
}

}  // namespace

hipError_t launch_experiment(int variant, const ChunkLaunch &a, bool verify, const uint32_t *tab,
                             const uint32_t *fold, int grid_cap, hipStream_t s) {
    switch (a.bpc) {
    case 512: return launch_exp_v<512>(variant, a, verify, tab, fold, grid_cap, s);
    case 1024: return launch_exp_v<1024>(variant, a, verify, tab, fold, grid_cap, s);
    case 2048: return launch_exp_v<2048>(variant, a, verify, tab, fold, grid_cap, s);
    case 4096: return launch_exp_v<4096>(variant, a, verify, tab, fold, grid_cap, s);
    case 8192: return launch_exp_v<8192>(variant, a, verify, tab, fold, grid_cap, s);
    case 16384: return launch_exp_v<16384>(variant, a, verify, tab, fold, grid_cap, s);
    case 65536: return launch_exp_v<65536>(variant, a, verify, tab, fold, grid_cap, s);
    default: return hipErrorInvalidValue;
    }
}

void set_variant(int v) { g_variant = v; }
void set_trace(uint64_t *d_trace) { g_trace = d_trace; }

hipError_t launch_stream_read(const uint8_t *d, uint64_t len, uint32_t *sink, int grid,
                              hipStream_t stream, bool overlap_previous) {
    // grid < 0: non-temporal loads over |grid| workgroups (the production kernels' policy);
    // overlap_previous: AQL packet without the barrier bit, as the overlapped verify launches
    const bool nt = grid < 0;
    const dim3 g(nt ? -grid : grid), b(256);
    auto k = nt ? stream_read_kernel<true> : stream_read_kernel<false>;
    if (overlap_previous)
        hipExtLaunchKernelGGL(k, g, b, 0, stream, nullptr, nullptr, hipExtAnyOrderLaunch, d, len / 16, sink);
    else
        hipLaunchKernelGGL(k, g, b, 0, stream, d, len / 16, sink);
    return hipGetLastError();
}

hipError_t launch_lane_read(const uint8_t *d, uint64_t len, uint32_t bpc, uint32_t *sink,
                            int grid_cap, hipStream_t stream) {
    const int variant = int(bpc >> 16);  // probe selector rides in the high bits of bpc
    bpc &= 0xFFFFu;
    const uint64_t chunks = len / bpc;
    const uint64_t lanes = variant == 2 ? chunks * 8 : variant == 3 ? chunks * 4 : chunks;
    const uint64_t need = (lanes + kBlockThreads - 1) / kBlockThreads;
    const int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
#define LR(B, V) hipLaunchKernelGGL((lane_read_kernel<B, V>), dim3(grid), dim3(kBlockThreads), 0, stream, d, chunks, sink)
#define LRV(B)                          \
    switch (variant) {                  \
    case 0: LR(B, 0); break;            \
    case 1: LR(B, 1); break;            \
    case 2: LR(B, 2); break;            \
    case 3: LR(B, 3); break;            \
    default: LR(B, 4); break;           \
    }
    switch (bpc) {
    case 512: LRV(512); break;
    case 2048: LRV(2048); break;
    case 4096: LRV(4096); break;
    default: return hipErrorInvalidValue;
    }
#undef LRV
#undef LR
    return hipGetLastError();
}

}  // namespace hdfs3crc
