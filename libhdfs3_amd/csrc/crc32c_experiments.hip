// Kernel variants kept for in-process A/B and diagnostics (hdfs3x_set_variant, tools/ab.py;
// docs/DESIGN_HISTORY.md §5.0), and the read-ceiling kernels of the bench. Linked into the measurement
// library libhdfs3_crc_lab.so only (HDFS3_LAB=1); the product libhdfs3_crc.so never sees it.
// Bit-exact variants are parity-tested (tests/test_gpu_parity.py); the diagnostic one gives
// wrong results on purpose. The designs that lost their A/B were removed in round 3; their
// numbers stay in docs/DESIGN_HISTORY.md §5 and profiles/.
#include "crc32c_wave.h"

namespace hdfs3crc {
namespace {

template <int BPC, bool V>
hipError_t launch_exp(int variant, const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                      hipStream_t s) {
    if constexpr (BPC > kRoundBytes) {
        if (variant == 115) return launch_r3<BPC, V, 1, true, true>(a, tab, fold, grid_cap, s);  // s_setprio
        if (variant == 123) return launch_r3<BPC, V, 1, true>(a, tab, fold, grid_cap, s);  // multi-round kernel
    }
    if constexpr (BPC <= kRoundBytes) {
        switch (variant) {
        case 92:  // production with the prefetch issued at the start of each step (early)
            return launch_wave3<BPC, V, false, true, kLabEarly>(a, tab, fold, grid_cap, s);
        case 93:  // production without the solo last step (overlapped verifies end interleaved)
            return launch_wave3<BPC, V, false, false>(a, tab, fold, grid_cap, s);
        case 94:  // the solo last step for overlapped verifies only (round-3 production before r3i)
            return launch_wave3<BPC, V, false, V>(a, tab, fold, grid_cap, s);
        case 95:  // compute at bpc 512 / 4096 without held stores (each round's words stored at once)
            return launch_wave3<BPC, V, false, true, kLabNoHold>(a, tab, fold, grid_cap, s);
        case 77:  // diagnostic: production with the table lookups replaced by an XOR (wrong results)
            return launch_wave3<BPC, V, false, true, kLabNoMath>(a, tab, fold, grid_cap, s);
        case 99:    // the pitch walk over this contiguous block as ONE packet (power-of-two rounds only)
        case 100: {  // the pitch walk over it as 8 equal packets (blocks of one 2-D tensor)
            const uint64_t units = a.len / kRoundBytes;
            const uint64_t npk = variant == 99 ? 1 : 8;
            const uint64_t upp = units / npk;
            if (a.len % kRoundBytes || units % npk || (upp & (upp - 1)) || a.chunk_base) return hipErrorInvalidValue;
            ChunkLaunch p = a;
            p.npk = npk;
            p.pitch = upp * kRoundBytes;
            p.crc_pitch = upp * (kRoundBytes / BPC) * 4;
            p.last_len = uint32_t(upp * kRoundBytes);
            if (!packet_geom(p.pitch, p.last_len, npk, BPC, &p.geom)) return hipErrorInvalidValue;
            return launch_wave3<BPC, V, true, false>(p, tab, fold, grid_cap, s);
        }
        case 115:  // s_setprio by rounds left at every launch size (production: waves of >= 16 rounds)
            return launch_wave3<BPC, V, false, true, kLabPrio>(a, tab, fold, grid_cap, s);
        case 117:  // no s_setprio at any size (production before r3y)
            return launch_wave3<BPC, V, false, true, kLabNoPrio>(a, tab, fold, grid_cap, s);
        case 118:  // diagnostic, compute: held words not stored (wrong results)
            return launch_wave3<BPC, V, false, true, kLabNoStore>(a, tab, fold, grid_cap, s);
        case 119:  // diagnostic, compute: held words stored over the wave's first round's words (wrong results)
            return launch_wave3<BPC, V, false, true, kLabNearStore>(a, tab, fold, grid_cap, s);
        case 123:  // (chunks above 4 KiB take the multi-round kernel; this size is production)
            return launch_wave3<BPC, V, false, true>(a, tab, fold, grid_cap, s);
        case 122:  // compute: held stores where production stages the words in LDS (before r3zb)
            return launch_wave3<BPC, V, false, true, kLabNoStage>(a, tab, fold, grid_cap, s);
        case 130:  // compute: staged words at every size, written out window by window (kLabStageWin)
            return launch_wave3<BPC, V, false, true, kLabStageWin>(a, tab, fold, grid_cap, s);
        case 157:  // the round-4 chains (16 table steps, the fold on the finished state; kLabFull16)
            return launch_wave3<BPC, V, false, true, kLabFull16>(a, tab, fold, grid_cap, s);
        case 128:  // compute: staged words through plain global stores (production before round 4)
            return launch_wave3<BPC, V, false, true, kLabStorePlain>(a, tab, fold, grid_cap, s);
        case 146:  // production with every wave's fill-done and first-data times (wave_spread.py --variant 146 --mid)
            return launch_wave3<BPC, V, false, true, kLabClock | kLabMid>(a, tab, fold, grid_cap, s);
        case 147:  // diagnostic: no table loads (wrong results), with fill-done / first-data stamps
            return launch_wave3<BPC, V, false, true, kLabNoTabLoad | kLabClock | kLabMid>(a, tab, fold, grid_cap, s);
        case 148:  // diagnostic: no table loads (wrong results)
            return launch_wave3<BPC, V, false, true, kLabNoTabLoad>(a, tab, fold, grid_cap, s);
        case 137:  // verify: 1024-thread workgroups at every launch size (production before round 4)
            return launch_wave3<BPC, V, false, true, kLabWg1024>(a, tab, fold, grid_cap, s);
        case 162:  // launches of <= 4096 units (16 MiB): one round per wave, twice the workgroups (round 6)
            return launch_wave3<BPC, V, false, true, kLabOneRound>(a, tab, fold, grid_cap, s);
        case 132:  // 256-thread workgroups (4 waves each): small launches spread over 4x the CUs
            return launch_wave3<BPC, V, false, true, 0, 256>(a, tab, fold, grid_cap, s);
        case 134:  // 512-thread workgroups (8 waves each)
            return launch_wave3<BPC, V, false, true, 0, 512>(a, tab, fold, grid_cap, s);
        case 125:  // production with clock stamps of workgroup 0 (kLabClock; tools/clock_ramp.py)
            return launch_wave3<BPC, V, false, true, kLabClock>(a, tab, fold, grid_cap, s);
        case 78:  // diagnostic: 77 without the slice-table LDS fill
            return launch_wave3<BPC, V, false, true, kLabNoMath | kLabNoFill>(a, tab, fold, grid_cap, s);
        default: return hipErrorInvalidValue;
        }
    }
    return hipErrorInvalidValue;
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

hipError_t lab_clock_buffer(unsigned long long *d, unsigned int cap, unsigned int *n_out) {
    // read the count of the previous buffer first, then install the new one with a zero count
    unsigned int n = 0;
    hipError_t e = hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_lab_clk_n), sizeof n);
    if (e != hipSuccess) return e;
    if (n_out) *n_out = n;
    const unsigned int zero = 0;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_lab_clk), &d, sizeof d)) != hipSuccess) return e;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_lab_clk_cap), &cap, sizeof cap)) != hipSuccess) return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_lab_clk_n), &zero, sizeof zero);
}

hipError_t lab_wave_buffer(unsigned long long *d, unsigned int cap, unsigned int *n_out) {
    // *n_out = launches stamped since the previous install; the launch counter restarts at 0
    if (n_out) *n_out = g_lab_seq.exchange(0);
    hipError_t e;
    const unsigned long long *none = nullptr;  // no stamps while the pair changes
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_lab_wave), &none, sizeof none)) != hipSuccess) return e;
    if (!d || !cap) return hipSuccess;
    if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_lab_wave_cap), &cap, sizeof cap)) != hipSuccess) return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_lab_wave), &d, sizeof d);
}

hipError_t launch_stream_read(const uint8_t *d, uint64_t len, uint32_t *sink, int grid,
                              hipStream_t stream, bool overlap_previous) {
    // grid < 0: non-temporal loads over |grid| workgroups (the production kernels' policy);
    // overlap_previous: AQL packet without the barrier bit, as the overlapped verify launches
    const bool nt = grid < 0;
    const dim3 g(nt ? -grid : grid), b(256);
    auto k = nt ? stream_read_kernel<true> : stream_read_kernel<false>;
    if (overlap_previous)
        hipExtLaunchKernelGGL(k, g, b, 0, stream, nullptr, nullptr, hipExtAnyOrderLaunch, d, len / 16, sink,
                              g_lab_seq++);
    else
        hipLaunchKernelGGL(k, g, b, 0, stream, d, len / 16, sink, g_lab_seq++);
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
