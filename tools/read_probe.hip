// HBM read-ceiling probe (measurement tool, not product): how fast can a read-only
// kernel stream 128 MiB per launch (bench shape: 8 rotating blocks, back-to-back
// launches on one stream) and 1 GiB per launch (steady state), by access pattern,
// grid, waves per CU, loads in flight and cache policy. Also the dependent-launch
// gap of empty kernels with and without a whole-CU LDS allocation.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/read_probe tools/read_probe.hip
//   tools/read_probe > gpurun_out/read_probe.jsonl
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
    if constexpr (NT) return __builtin_nontemporal_load(q);
    return *q;
}
// one 4 KiB round through a buffer resource built from the wave-uniform base: the lane
// offset is the only VGPR operand (no VGPR address temporaries for the allocator to alias
// with in-flight destinations, which makes the waitcnt pass drain at the loop head)
template <bool NT>
__device__ __forceinline__ void ld_round(u32x4 (&r)[4], const uint8_t *base, uint32_t lane_off) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(b));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(b >> 32));
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>((uint64_t(hi) << 32) | lo), 0, 4096, 0x00020000);
#pragma unroll
    for (int t = 0; t < 4; ++t) r[t] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + 1024 * t, 0, NT ? 2 : 0);
}
__device__ __forceinline__ uint32_t fold(u32x4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// grid-stride: lane i reads 16 B at i, i+S, ..., U loads in flight per iteration
template <int U, bool NT>
__global__ void k_stride(const uint8_t *__restrict__ d, uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    const uint64_t S = uint64_t(gridDim.x) * blockDim.x;
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * S < n16; i += U * S) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(d + 16 * (i + u * S));
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= fold(v[u]);
    }
    for (; i < n16; i += S) acc ^= fold(ld<NT>(d + 16 * i));
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// rounds: wave w reads 4 KiB rounds w, w+W, w+2W, ... (4 x 1 KiB coalesced loads per
// round), D rounds in flight. MODE 0: round-robin; 1: each wave a contiguous span of
// rounds; 2: XCD-aware round-robin (blockIdx -> XCD is blockIdx % 8: wave groups of
// one XCD take consecutive rounds of the same window).
template <int D, bool NT, int MODE>
__global__ __launch_bounds__(D >= 8 ? 512 : 1024) void k_rounds(const uint8_t *__restrict__ d, uint64_t len, uint32_t *sink) {
    extern __shared__ uint32_t lds_pad[];
    const uint64_t nunits = len / 4096;
    const uint32_t wpb = blockDim.x / 64;
    const uint64_t W = uint64_t(gridDim.x) * wpb;
    uint64_t wave = uint64_t(blockIdx.x) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr (MODE == 2 || MODE == 3) {
        const uint32_t nb = gridDim.x, x = blockIdx.x % 8, b = blockIdx.x / 8;
        const uint32_t per = nb / 8;
        wave = (uint64_t(x) * per + b) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    }
    const uint32_t lane = threadIdx.x & 63;
    uint64_t k0, kn, step;
    if constexpr (MODE == 1) {
        const uint64_t per = (nunits + W - 1) / W;
        k0 = wave * per;
        kn = k0 + per < nunits ? k0 + per : nunits;
        step = 1;
    } else if constexpr (MODE == 3) {
        // XCD-blocked: XCD x owns the contiguous eighth [x*n/8, (x+1)*n/8) of the buffer,
        // its waves round-robin over it
        const uint64_t wx = W / 8, x = blockIdx.x % 8, wi = wave - x * wx;
        const uint64_t per = nunits / 8;
        k0 = x * per + wi;
        kn = (x + 1) * per;
        step = wx;
    } else {
        k0 = wave;
        kn = nunits;
        step = W;
    }
    // loads stay unconditional (a guarded load makes the waitcnt pass drain at the
    // loop head): past the wave's end they read the cache-resident 4 KiB `dummy`
    const uint8_t *dummy = reinterpret_cast<const uint8_t *>(sink) + 4096;
    auto src = [&](uint64_t kk) { return kk < kn ? d + kk * 4096 : dummy; };
    uint32_t acc = 0;
    u32x4 b[D][4];
    uint64_t k = k0;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        ld_round<NT>(b[i], src(k + i * step), 16 * lane);
        __builtin_amdgcn_sched_barrier(0);
    }
    for (; k < kn; k += D * step) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const uint64_t kk = k + i * step;
            uint32_t x = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) x ^= fold(b[i][t]);
            acc ^= kk < kn ? x : 0u;
            __builtin_amdgcn_sched_barrier(0);
            ld_round<NT>(b[i], src(kk + D * step), 16 * lane);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc + lds_pad[0];
}

// rounds_rr with synthetic per-round work on the round's words: VALU ops (v_perm/xor
// chains, 4 independent accumulators) and conflict-free LDS reads (own-bank words)
template <int D, int NV, int NL>
__global__ __launch_bounds__(1024) void k_rounds_work(const uint8_t *__restrict__ d, uint64_t len, uint32_t *sink) {
    extern __shared__ uint32_t lds_pad[];
    const uint64_t nunits = len / 4096;
    const uint32_t wpb = blockDim.x / 64;
    const uint64_t W = uint64_t(gridDim.x) * wpb;
    const uint64_t wave = uint64_t(blockIdx.x) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < 8192; i += blockDim.x) lds_pad[i] = i * 0x9E3779B9u;
    __syncthreads();
    const uint8_t *dummy = reinterpret_cast<const uint8_t *>(sink) + 4096;
    auto src = [&](uint64_t kk) { return kk < nunits ? d + kk * 4096 : dummy; };
    uint32_t acc[4] = {0, 1, 2, 3};
    u32x4 b[D][4];
    uint64_t k = wave;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        ld_round<true>(b[i], src(k + i * W), 16 * lane);
        __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t lbase = (lane & 31) * 4;
    for (; k < nunits; k += D * W) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const uint64_t kk = k + i * W;
            uint32_t x[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) x[t] = fold(b[i][t]);
            __builtin_amdgcn_sched_barrier(0);
            ld_round<true>(b[i], src(kk + D * W), 16 * lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int n = 0; n < NV / 4; ++n)
#pragma unroll
                for (int t = 0; t < 4; ++t) x[t] = __builtin_amdgcn_perm(x[t], x[(t + 1) & 3] ^ n, 0x05040100u + n);
#pragma unroll
            for (int n = 0; n < NL / 4; ++n)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    x[t] ^= lds_pad[(((x[t] >> 8) & 0xFFu) * 32 * 4 + lbase) / 4 + (n & 3) * 8192 / 4 / 4];
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] ^= kk < nunits ? x[t] : 0u;
        }
    }
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9E3779B9u) sink[0] = 1;
}

// LDS read throughput: every wave issues N conflict-free reads of width B bytes per lane
// (addresses from a per-lane LCG, rounded to the lane's own bank group), 8 independent
// accumulators so latency is hidden; 256 workgroups x 1024 threads, 160 KiB LDS.
template <int B, int N>
__global__ __launch_bounds__(1024) void k_lds(uint32_t *sink) {
    extern __shared__ uint32_t lds[];
    for (uint32_t i = threadIdx.x; i < 160 * 1024 / 4; i += blockDim.x) lds[i] = i * 0x9E3779B9u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    // lanes of a half-wave cover all 32 banks; unrolled reads differ only in the immediate
    // offset (rows 16 apart), so the loop is ~1 VALU per read (the xor consuming it)
    constexpr uint32_t kRow = 32 * B;
    uint32_t base = (lane & 31) * B + (threadIdx.x >> 6) * kRow;
    uint32_t acc0 = 0, acc1 = 0;
    const uint8_t *l8 = reinterpret_cast<const uint8_t *>(lds);
    for (int it = 0; it < N / 16; ++it) {
#pragma unroll
        for (int a = 0; a < 16; ++a) {
            const uint8_t *p = l8 + base + a * 16 * kRow;
            if constexpr (B == 4) {
                uint32_t v;  // asm: keep single ds_read_b32 (the compiler pairs plain loads into read2)
                asm volatile("ds_read_b32 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(8)" : "=v"(v) : "v"(base), "i"(a * 16 * kRow & 0xFFFF));
                acc0 ^= v;
                (void)p;
            } else if constexpr (B == 8) {
                const uint2 v = *reinterpret_cast<const uint2 *>(p);
                acc0 ^= v.x;
                acc1 ^= v.y;
            } else {
                const uint4 v = *reinterpret_cast<const uint4 *>(p);
                acc0 ^= v.x ^ v.z;
                acc1 ^= v.y ^ v.w;
            }
        }
        base = (base + 3 * kRow) & (32 * 1024 - 1);
    }
    if ((acc0 ^ acc1) == 0x9E3779B9u) sink[0] = 1;
}

// rounds_rr with NG L1-resident gathers per round: dword loads at data-derived offsets in
// a 4 KiB table image (buffer descriptor, lane-varying offset), issued BEFORE the round's
// prefetch (so in-order vmcnt never makes them wait for HBM) and consumed after it.
template <int NG>
__global__ __launch_bounds__(1024) void k_rounds_gather(const uint8_t *__restrict__ d, uint64_t len,
                                                       const uint32_t *__restrict__ tab, uint32_t *sink) {
    extern __shared__ uint32_t lds_pad[];
    constexpr int D = 2;
    const uint64_t nunits = len / 4096;
    const uint64_t W = uint64_t(gridDim.x) * 16;
    const uint64_t wave = uint64_t(blockIdx.x) * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint8_t *dummy = reinterpret_cast<const uint8_t *>(sink) + 4096;
    auto src = [&](uint64_t kk) { return kk < nunits ? d + kk * 4096 : dummy; };
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(tab), 0, 4096, 0x00020000);
    uint32_t acc = 0;
    u32x4 b[D][4];
    uint64_t k = wave;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        ld_round<true>(b[i], src(k + i * W), 16 * lane);
        __builtin_amdgcn_sched_barrier(0);
    }
    for (; k < nunits; k += D * W) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const uint64_t kk = k + i * W;
            uint32_t x[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) x[t] = fold(b[i][t]);
            uint32_t g[NG > 0 ? NG : 1];
#pragma unroll
            for (int n = 0; n < NG; ++n)
                g[n] = __builtin_amdgcn_raw_buffer_load_b32(
                    trs, ((x[n & 3] >> (8 * ((n >> 2) & 3))) & 0xFFu) * 4 + ((n >> 4) & 3) * 1024, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            ld_round<true>(b[i], src(kk + D * W), 16 * lane);
            __builtin_amdgcn_sched_barrier(0);
            uint32_t y = x[0] ^ x[1] ^ x[2] ^ x[3];
#pragma unroll
            for (int n = 0; n < NG; ++n) y ^= g[n];
            acc ^= kk < nunits ? y : 0u;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc + lds_pad[0];
}

__global__ void k_empty(uint32_t *sink) {
    extern __shared__ uint32_t lds_pad[];
    if (threadIdx.x == 0 && blockIdx.x == 0 && sink[1] == 0x12345678u) sink[0] = lds_pad[0];
}

struct Res {
    double us_launch_128;  // per launch, 100 back-to-back 128 MiB launches over 8 rotating slices
    double us_1g;          // median single 1 GiB launch
};

static uint8_t *g_buf;
static uint32_t *g_sink;
static hipStream_t g_st;
// mode 6: launches after the first of each back-to-back batch go out without the AQL barrier bit
// (hipExtAnyOrderLaunch, as the CRC kernels' HDFS3_LAUNCH_OVERLAP_PREVIOUS)
static bool g_overlap = false, g_ovl_now = false;
template <typename K, typename... A>
static void launch_k(K k, dim3 g, dim3 b, size_t lds, A... a) {
    if (g_ovl_now)
        hipExtLaunchKernelGGL(k, g, b, lds, g_st, nullptr, nullptr, hipExtAnyOrderLaunch, a...);
    else
        hipLaunchKernelGGL(k, g, b, lds, g_st, a...);
}
static const uint64_t kBlk = 128ull << 20, kAll = 1ull << 30;

template <typename F>
static Res measure(F launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 10; ++i) {
        g_ovl_now = g_overlap && i > 0;
        launch(g_buf + (i % 8) * kBlk, kBlk);
    }
    CK(hipStreamSynchronize(g_st));
    const int K = 100;
    CK(hipEventRecord(e0, g_st));
    for (int i = 0; i < K; ++i) {
        g_ovl_now = g_overlap && i > 0;
        launch(g_buf + (i % 8) * kBlk, kBlk);
    }
    g_ovl_now = false;
    CK(hipEventRecord(e1, g_st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    Res r;
    r.us_launch_128 = 1000.0 * ms / K;
    std::vector<double> v;
    for (int i = 0; i < 9; ++i) {
        CK(hipEventRecord(e0, g_st));
        launch(g_buf, kAll);
        CK(hipEventRecord(e1, g_st));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.push_back(1000.0 * ms);
    }
    std::sort(v.begin(), v.end());
    r.us_1g = v[v.size() / 2];
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return r;
}

static void report(const char *kind, int grid, int block, int depth, int nt, int lds_kib, Res r) {
    printf("{\"kernel\": \"%s\", \"grid\": %d, \"block\": %d, \"depth\": %d, \"nt\": %d, \"lds_kib\": %d, "
           "\"us_per_launch_128MiB\": %.2f, \"GBps_128MiB\": %.1f, \"us_1GiB\": %.2f, \"GBps_1GiB\": %.1f}\n",
           kind, grid, block, depth, nt, lds_kib, r.us_launch_128, kBlk / r.us_launch_128 / 1e3, r.us_1g,
           kAll / r.us_1g / 1e3);
    fflush(stdout);
}

template <int U, bool NT>
static void run_stride(int grid, int block) {
    Res r = measure([&](const uint8_t *p, uint64_t n) {
        launch_k(k_stride<U, NT>, dim3(grid), dim3(block), 0, p, n / 16, g_sink);
    });
    report(g_overlap ? "stride_ovl" : "stride", grid, block, U, NT, 0, r);
}

template <int D, bool NT, int MODE>
static void run_rounds(int grid, int block, int lds_kib) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rounds<D, NT, MODE>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, lds_kib * 1024));
    Res r = measure([&](const uint8_t *p, uint64_t n) {
        launch_k(k_rounds<D, NT, MODE>, dim3(grid), dim3(block), lds_kib * 1024, p, n, g_sink);
    });
    static const char *names[] = {"rounds_rr", "rounds_contig", "rounds_xcd", "rounds_xcdblk"};
    static const char *onames[] = {"rounds_rr_ovl", "rounds_contig_ovl", "rounds_xcd_ovl", "rounds_xcdblk_ovl"};
    report(g_overlap ? onames[MODE] : names[MODE], grid, block, D, NT, lds_kib, r);
}

template <int D, int NV, int NL>
static void run_work(int lds_kib) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rounds_work<D, NV, NL>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, lds_kib * 1024));
    Res r = measure([&](const uint8_t *p, uint64_t n) {
        hipLaunchKernelGGL((k_rounds_work<D, NV, NL>), dim3(256), dim3(1024), lds_kib * 1024, g_st, p, n, g_sink);
    });
    char name[64];
    snprintf(name, sizeof name, "work_v%d_l%d", NV, NL);
    report(name, 256, 1024, D, 1, lds_kib, r);
}

template <int B, int N>
static void run_lds() {
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_lds<B, N>), hipFuncAttributeMaxDynamicSharedMemorySize,
                           160 * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_lds<B, N>), dim3(256), dim3(1024), 160 * 1024, g_st, g_sink);
    CK(hipEventRecord(e0, g_st));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k_lds<B, N>), dim3(256), dim3(1024), 160 * 1024, g_st, g_sink);
    CK(hipEventRecord(e1, g_st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / 5;
    // per CU: 16 waves x N wave-instructions
    printf("{\"kernel\": \"lds_read_b%d\", \"reads_per_wave\": %d, \"us\": %.2f, \"ns_per_wave_instr_per_cu\": %.3f, "
           "\"GBps_chip\": %.0f}\n",
           8 * B, N, us, us * 1000.0 / (16.0 * N), 256.0 * 16 * N * 64.0 * B / (us * 1e3));
    fflush(stdout);
}

template <int NG>
static void run_gather() {
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rounds_gather<NG>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const uint32_t *tab = g_sink + 2048;  // bytes 8 KiB.. of the sink buffer
    Res r = measure([&](const uint8_t *p, uint64_t n) {
        hipLaunchKernelGGL((k_rounds_gather<NG>), dim3(256), dim3(1024), 160 * 1024, g_st, p, n, tab, g_sink);
    });
    char name[64];
    snprintf(name, sizeof name, "gather_%d", NG);
    report(name, 256, 1024, 2, 1, 160, r);
}

static void run_empty(int grid, int block, int lds_kib) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_empty), hipFuncAttributeMaxDynamicSharedMemorySize,
                           lds_kib * 1024));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(block), lds_kib * 1024, g_st, g_sink);
    const int K = 200;
    CK(hipEventRecord(e0, g_st));
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(block), lds_kib * 1024, g_st, g_sink);
    CK(hipEventRecord(e1, g_st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"empty\", \"grid\": %d, \"block\": %d, \"lds_kib\": %d, \"us_per_launch\": %.2f}\n", grid,
           block, lds_kib, 1000.0 * ms / K);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    CK(hipStreamCreateWithFlags(&g_st, hipStreamNonBlocking));
    CK(hipMalloc(&g_buf, kAll));
    CK(hipMalloc(&g_sink, 16384));
    CK(hipMemset(g_buf, 0x5A, kAll));
    CK(hipMemset(g_sink, 0, 16384));
    CK(hipDeviceSynchronize());

    if (only < 0 || only == 0) {
        run_empty(1, 64, 0);
        run_empty(256, 1024, 0);
        run_empty(256, 1024, 160);
        run_empty(1024, 256, 0);
    }
    if (only < 0 || only == 1) {
        for (int g : {256, 512, 768, 1024, 2048, 4096}) run_stride<4, false>(g, 256);
        for (int g : {256, 512, 1024, 2048}) run_stride<4, true>(g, 256);
        for (int g : {256, 512, 1024}) run_stride<8, false>(g, 256);
        for (int g : {256, 512}) run_stride<4, false>(g, 1024);
        for (int g : {256, 512}) run_stride<8, false>(g, 512);
    }
    if (only < 0 || only == 2) {
        for (int rep = 0; rep < 3; ++rep) {
            run_rounds<1, true, 0>(256, 1024, 160);
            run_rounds<2, true, 0>(256, 1024, 160);
            run_rounds<3, true, 0>(256, 1024, 160);
            run_rounds<1, true, 2>(256, 1024, 160);
            run_rounds<2, true, 2>(256, 1024, 160);
            run_rounds<3, true, 2>(256, 1024, 160);
            run_rounds<1, true, 3>(256, 1024, 160);
            run_rounds<2, true, 3>(256, 1024, 160);
            run_rounds<2, true, 0>(256, 768, 160);
            run_rounds<3, true, 0>(256, 768, 160);
            run_rounds<2, true, 0>(256, 512, 160);
            run_rounds<4, true, 0>(256, 512, 160);
            run_rounds<2, false, 0>(256, 1024, 160);
            run_stride<4, true>(512, 256);
        }
    }
    if (only == 3) {
        for (int rep = 0; rep < 3; ++rep) {
            run_rounds<2, true, 0>(256, 1024, 160);
            run_work<2, 0, 0>(160);
            run_work<2, 64, 0>(160);
            run_work<2, 128, 0>(160);
            run_work<2, 192, 0>(160);
            run_work<2, 0, 64>(160);
            run_work<2, 0, 128>(160);
            run_work<2, 128, 64>(160);
        }
    }
    if (only == 4) {
        for (int rep = 0; rep < 2; ++rep) {
            run_lds<4, 4096>();
            run_lds<8, 4096>();
            run_lds<16, 4096>();
            run_lds<4, 16384>();
            run_lds<8, 16384>();
        }
    }
    if (only == 5) {
        for (int rep = 0; rep < 3; ++rep) {
            run_rounds<2, true, 0>(256, 1024, 160);
            run_gather<0>();
            run_gather<8>();
            run_gather<16>();
            run_gather<32>();
            run_work<2, 0, 32>(160);
        }
    }
    if (only == 6) {  // co-residency: the CRC geometry (1 workgroup/CU) against 2 per CU, both launch modes
        for (int rep = 0; rep < 3; ++rep) {
            for (bool ov : {false, true}) {
                g_overlap = ov;
                run_rounds<2, true, 0>(256, 1024, 160);
                run_rounds<2, true, 0>(256, 1024, 80);
                run_rounds<2, true, 0>(512, 1024, 80);
                run_rounds<2, true, 0>(512, 512, 80);
                run_rounds<2, true, 0>(256, 1024, 0);
                run_stride<4, true>(512, 256);
                run_stride<4, false>(512, 256);
            }
            g_overlap = false;
        }
    }
    if (only == 7) {  // in flight per CU: waves per CU x rounds in flight, 1 workgroup per CU (160 KiB)
        for (int rep = 0; rep < 3; ++rep) {
            for (bool ov : {false, true}) {
                g_overlap = ov;
                run_rounds<1, true, 0>(256, 1024, 160);
                run_rounds<2, true, 0>(256, 1024, 160);
                run_rounds<2, true, 0>(256, 768, 160);
                run_rounds<2, true, 0>(256, 512, 160);
                run_rounds<3, true, 0>(256, 512, 160);
                run_rounds<4, true, 0>(256, 512, 160);
                run_rounds<2, true, 0>(256, 256, 160);
                run_rounds<4, true, 0>(256, 256, 160);
                run_stride<4, true>(512, 256);
            }
            g_overlap = false;
        }
    }
    CK(hipFree(g_buf));
    CK(hipFree(g_sink));
    return 0;
}
