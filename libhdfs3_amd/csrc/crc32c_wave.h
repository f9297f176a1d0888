// The production round kernel (bpc 512 / 1024 / 2048 / 4096) of libhdfs3's per-chunk
// CRC32C: verify-on-read (RemoteBlockReader::verifyChecksum, src/client/RemoteBlockReader.cpp:306-326;
// LocalBlockReader::readAndVerify, src/client/LocalBlockReader.cpp:138-163) and compute-on-write
// (OutputStreamImpl::appendInternal, src/client/OutputStreamImpl.cpp:298-359) over a whole block,
// a constant-pitch packet stream or a list of segments in one launch. Internal; not installed.
//
// Work unit: a ROUND = 4 KiB of contiguous data, one wave at a time (crc32c_device.h: load_round_buf,
// regroup, Lut, fold_half, group_xor). A wave consumes two rounds per STEP as two software-pipelined
// lookup chains and has the next step's two rounds in flight while it does (8 KiB per wave, 128 KiB
// per CU). The round -> data mapping is a WALK:
//   BlockWalk   one contiguous block (unit u at data + 4096 u);
//   PitchWalk   a packet stream at a constant pitch, or equal blocks of one 2-D tensor
//               (unit u = round u % upp of packet u / upp; a packet's last round may be partial);
//   SegWalk     a list of independent segments (ragged batches, packets in descriptor lists),
//               the prefetch stream's current segment cached in scalar registers.
// Every view a walk returns (data pointer, the round's CRC-word pointer, the key of its first chunk)
// is wave-uniform, so its arithmetic is SALU and the word loads/stores take the saddr form.
//
// Loop shape (round 3). The buffers rotate A -> B -> A by unrolling; every step in a loop is the same
// code, and whatever follows a loop reads only ONE buffer set. The round-2 kernel left its loop from
// the middle of the body into two inlined tails, one per buffer set; the register allocator then kept
// the second step's rounds in two places and copied them (32 v_mov per step) and drained every load
// at the loop head (vmcnt(0)). Overlapped verifies end with a solo last step after the loop, on the
// buffer set fixed by the parity of the wave's step count (two copies of the loop, wave_rounds).
#pragma once

#include "crc32c_device.h"

namespace hdfs3crc {
namespace {

// Lab-only bits of the round kernel (crc32c_experiments.hip; production passes 0):
constexpr int kLabEarly = 1;   // prefetch issued at the start of each step, not after its rounds landed
constexpr int kLabNoMath = 2;  // diagnostic: table lookups replaced by an XOR of the words (wrong results)
constexpr int kLabNoHold = 4;  // compute at bpc 512 / 4096: store each round's words at once (no held stores)
constexpr int kLabNoFill = 8;  // diagnostic: the slice tables are not written to LDS (wrong results)
constexpr int kLabPrio = 16;    // s_setprio by rounds left at every launch size (production: >= kPrioMinRounds)
constexpr int kLabNoPrio = 32;  // no s_setprio at any launch size (the round-3 production before r3y)
constexpr int kLabNoStore = 64;     // diagnostic, compute: the held words are not stored (wrong results)
constexpr int kLabNearStore = 128;  // diagnostic, compute: every flush stores to the wave's first round's words
constexpr int kLabNoStage = 1024;   // compute: held stores even where production stages the words (kStageWords)
constexpr int kLabStageWin = 2048;  // compute at bpc 512: staged words past kStageMaxRounds too, window by window
constexpr int kLabClock = 4096;     // clock stamps of workgroup 0 (LabClock, crc32c_device.h; lab builds only)
constexpr int kLabStorePlain = 8192;  // compute, staged words: plain global stores (production before round 4)
constexpr int kLabWg1024 = 16384;    // verify: 1024-thread workgroups at every launch size (production before round 4)
constexpr int kLabNoTabLoad = 2097152;  // diagnostic: the table images are not loaded (made up from t: wrong results)
constexpr int kLabFull16 = 8388608;  // the round-4 chains: 16 table steps per chain, the fold on the finished state
constexpr int kLabOneRound = 4194304;  // launches of <= 4096 units: one round per wave (twice the workgroups)
constexpr int kLabMid = 1048576;     // with kLabClock: word 2 of a wave's stamp = fill done | first data << 21 | kernel
                                     // arguments landed << 42, each - start, 21 bits of 10 ns
// Not a lab bit: launch_wave3 sets it for compute over a contiguous block at bpc 1024 / 2048, and at
// bpc 512 when its waves have at most kStageMaxRounds(512) rounds (the words are staged in LDS and
// written as whole lines, §4.1; past the window size in windows)
constexpr int kStageWords = 512;
// 16 waves x R rounds x (4096 / bpc) words = the 4096 words (16 KiB) the half fold image leaves:
// 32 rounds at bpc 512, 64 at 1024, 128 at 2048
constexpr uint32_t kStageMaxRounds(int bpc) { return uint32_t(bpc / 16); }

// Waves with at least this many rounds set their priority by the rounds they have left (round 3):
// the SIMD arbiter favours older waves, so with equal work a workgroup's waves end staggered and its
// last ones run nearly alone, too few to keep the CU's share of HBM busy. With priority 3..0 by the
// quartile of rounds left the lagging waves catch up and the workgroup drains together: 1 GiB per
// launch 168.8 -> 162.5 us barriered, 161.9 -> 157.4 overlapped, the batch API (8 x 128 MiB) 167.1 ->
// 161.0, compute 171.0 -> 163.8; 256 MiB -1.9 % / -1.0 %. At 128 MiB (8 rounds per wave) it costs
// 0.2-0.7 us, so short waves keep the arbiter's order (profiles/r03/reentry/r3x_ab_*, r3y_*).
constexpr uint32_t kPrioMinRounds = 16;

typedef __attribute__((address_space(1))) const uint32_t gcu32;
typedef __attribute__((address_space(1))) const uint8_t gcu8;
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(4))) const SegLaunch CSegLaunch;
typedef __attribute__((address_space(4))) const DevSegment CDevSegment;

// A round's view: data, CRC words of its first chunk (stored words when verifying, the output when
// computing), result key of its first chunk, valid bytes (4096, or the whole chunks of a partial
// last round of a packet or segment: PacketGeom).
struct WView {
    const uint8_t *p;
    uint8_t *w;
    uint64_t key;
    uint32_t nb;
};

// Rounds of one contiguous block: the wave's rounds are units wave, wave + W, ... (W = waves).
// kLaneView: view() also takes a lane-varying round index (the held compute stores find their
// words' addresses at flush time); a walk without it holds each word's address instead.
template <int CPU>
struct BlockWalk {
    static constexpr bool kLaneView = true;
    static constexpr bool kContiguous = true;  // unit u's words at words + 4 * CPU * u
    const uint8_t *data;
    uint8_t *words;
    uint64_t key0, first, stride;
    uint32_t K;            // rounds of this wave (< 2^32: 16 TiB per launch); 32-bit so k < K is SALU
    const uint8_t *dummy;  // the cache-resident 4 KiB table image: reads past the wave's last round
    uint32_t kq = 0, kr = 0;  // the launch's round split (ChunkLaunch::kq/kr): any wave's K
    __device__ __forceinline__ WView view(uint32_t k) const {
        const uint64_t u = first + uint64_t(k) * stride;
        const bool in = k < K;
        return WView{in ? data + u * kRoundBytes : dummy, in ? words + 4 * CPU * u : const_cast<uint8_t *>(dummy),
                     key0 + CPU * u, uint32_t(kRoundBytes)};
    }
};

// A packet stream at one pitch (PacketGeom): every packet but the last holds upp units, the last
// lunits; a packet's last unit holds ptail (the last packet: ltail) valid bytes. Its words sit at
// words + packet * wpitch (the wire layout: in the packet; the writer's batches and a [blocks,
// words] tensor: their own pitch). Keys are (packet << 32) | chunk. Unit indices stay below 2^31
// (the host's packet_geom), so the packet is a 32 x 32 multiply-shift: SALU for the wave's own
// views, VALU only for the held stores' lane-varying ones.
template <int CPU>
struct PitchWalk {
    static constexpr bool kLaneView = true;
    static constexpr bool kContiguous = false;
    const uint8_t *data;
    uint8_t *words;
    uint64_t dpitch, wpitch, first, stride;
    uint32_t K;
    uint32_t upp, magic, shift, ptail, lunits, ltail, lpk;
    const uint8_t *dummy;
    __device__ __forceinline__ WView view(uint32_t k) const {
        const uint32_t u = uint32_t(first + uint64_t(k) * stride);
        const uint32_t pk = uint32_t((uint64_t(u) * magic) >> shift), r = u - pk * upp;
        const bool lastp = pk == lpk;
        const uint32_t nb = r + 1 == (lastp ? lunits : upp) ? (lastp ? ltail : ptail) : uint32_t(kRoundBytes);
        const bool in = k < K;
        return WView{in ? data + uint64_t(pk) * dpitch + uint64_t(r) * kRoundBytes : dummy,
                     in ? words + uint64_t(pk) * wpitch + 4 * CPU * r : const_cast<uint8_t *>(dummy),
                     (uint64_t(pk) << 32) | (CPU * r), in ? nb : uint32_t(kRoundBytes)};
    }
};

// The union of a list of independent segments' whole rounds (SegLaunch, crc32c_device.h): global
// unit u belongs to the segment with the largest unit_begin <= u, found as u / uniform when the host
// found equal segments (UNI), else by a wave-uniform binary search over the descriptors. The prefetch
// stream's current segment is cached in scalar registers, so a round inside it costs arithmetic only
// and crossing into another one a lookup and its scalar descriptor loads. Views are asked for in
// increasing round order (the core resolves the next step's views at the end of each step).
template <int CPU, bool UNI>
struct SegWalk {
    static constexpr bool kLaneView = false;
    static constexpr bool kContiguous = false;
    // The launch record and the descriptors through the CONSTANT address space: their fields are
    // wave-uniform, so they load with s_load (lgkmcnt). Through a generic pointer they compiled to
    // FLAT loads, which count on vmcnt as well, and every segment crossing then waited for the whole
    // prefetch stream (vmcnt(0)) before it could resolve the next view.
    CSegLaunch *L;
    uint64_t first, stride;
    uint32_t K;
    const uint8_t *dummy;
    uint64_t c_begin = 1, c_end = 0, c_key = 0;
    uint64_t c_wlen = 0;  // the cached segment's whole-chunk bytes (its last unit may be partial)
    const uint8_t *c_data = nullptr;
    uint8_t *c_crc = nullptr;
    uint32_t c_si = ~0u;  // index of the cached segment (~0: none yet)
    static constexpr uint32_t kBpc = uint32_t(kRoundBytes / CPU);

    __device__ __forceinline__ static uint64_t wlen(uint64_t len) { return len / kBpc * kBpc; }
    __device__ __forceinline__ static uint64_t units(uint64_t len) { return (wlen(len) + kRoundBytes - 1) / kRoundBytes; }
    __device__ __forceinline__ CDevSegment *segp(uint32_t i) const {
        return L->seg ? (CDevSegment *)(L->seg) + i : L->inl + i;
    }
    __device__ __forceinline__ uint32_t seg_of(uint64_t u) const {
        if constexpr (UNI) {  // unit counts stay < 2^32 (16 TiB per launch): 32-bit divide
            const uint32_t si = uint32_t(u) / uint32_t(L->uniform);
            return si < L->nseg ? si : L->nseg - 1;
        } else {
            uint32_t lo = 0, hi = L->nseg - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (rfl64(segp(mid)->unit_begin) <= u) lo = mid;
                else hi = mid - 1;
            }
            return lo;
        }
    }
    __device__ __forceinline__ WView view(uint32_t k) {
        if (k >= K) return WView{dummy, const_cast<uint8_t *>(dummy), 0, uint32_t(kRoundBytes)};
        const uint64_t u = first + uint64_t(k) * stride;
        if (u < c_begin || u >= c_end) {
            uint32_t si;
            if constexpr (UNI) {
                si = seg_of(u);
            } else {
                // the walk only moves forward, and with segments longer than the walk's stride it
                // lands in the next one: try that first (one descriptor load, which the view needs
                // anyway), then the unit map of a long list (one load), else the binary search (a chain
                // of dependent loads)
                const uint32_t nx = c_si + 1;
                if (nx < L->nseg && u >= rfl64(segp(nx)->unit_begin) &&
                    u < rfl64(segp(nx)->unit_begin) + units(rfl64(segp(nx)->len)))
                    si = nx;
                else if (L->unit_seg)
                    si = __builtin_amdgcn_readfirstlane(
                        ((__attribute__((address_space(4))) const uint32_t *)(L->unit_seg))[u]);
                else
                    si = seg_of(u);
            }
            if (L->stride) {  // packets at one pitch: kernel-argument arithmetic, no descriptor loads
                const bool lastp = si + 1 >= L->nseg;
                c_begin = uint64_t(si) * L->uniform;
                c_wlen = wlen(lastp ? L->inl[1].len : L->inl[0].len);
                c_end = c_begin + (lastp ? units(L->inl[1].len) : L->uniform);
                c_data = L->inl[0].data + uint64_t(si) * L->stride;
                c_crc = L->dense_words ? L->dense_words + 4 * CPU * c_begin : L->inl[0].crc + uint64_t(si) * L->stride;
                c_key = uint64_t(si) << 32;
            } else {
                CDevSegment *sd = segp(si);
                c_begin = rfl64(sd->unit_begin);
                c_wlen = wlen(rfl64(sd->len));
                c_end = c_begin + (c_wlen + kRoundBytes - 1) / kRoundBytes;
                c_data = reinterpret_cast<const uint8_t *>(rfl64(reinterpret_cast<uint64_t>(sd->data)));
                c_crc = L->dense_words ? L->dense_words + 4 * CPU * c_begin
                                       : reinterpret_cast<uint8_t *>(rfl64(reinterpret_cast<uint64_t>(sd->crc)));
                c_key = rfl64(sd->key_base);
            }
            c_si = si;
        }
        const uint64_t r = u - c_begin, left = c_wlen - r * kRoundBytes;
        return WView{c_data + r * kRoundBytes, c_crc + 4 * CPU * r, c_key + CPU * r,
                     left < kRoundBytes ? uint32_t(left) : uint32_t(kRoundBytes)};
    }
};

// The core: prologue, steps, last step. VERIFY: compare with the stored words and fold the first bad
// key into *result; else store the words. SOLO (overlapped verifies): the last step runs its two
// rounds as single chains one after the other. HOLD (compute, bpc 512): the words of 8 rounds are
// transposed into one VGPR and up to 8 such VGPRs are stored in one burst. LAB: lab-only bits (kLab*).
template <int BPC, bool VERIFY, bool SOLO, bool HOLD, int LAB, int TPB, class Walk>
__device__ __forceinline__ void wave_rounds(Walk &walk, uint32_t *lds, const uint32_t *__restrict__ g_tab,
                                            const uint32_t *__restrict__ g_nib, unsigned long long *result,
                                            unsigned long long *lab_mid = nullptr) {
    constexpr int G = BPC / 64;
    constexpr bool kHalfFold = G <= 32;
    constexpr bool LATE = (LAB & kLabEarly) == 0, NOMATH = (LAB & kLabNoMath) != 0;
    constexpr bool kWrong = (LAB & (kLabNoMath | kLabNoFill | kLabNoTabLoad)) != 0;  // diagnostics: wrong CRCs (verify)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane % G;
    const uint32_t lane_off = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint32_t K = walk.K;

    // lean fill: each of the image's 1024 slice-table words replicated 32x (TPB threads take 1024 / TPB
    // words each); for G <= 32 the half fold image
    constexpr int kFillIters = 1024 / TPB;
    static_assert(kFillIters * TPB == 1024, "TPB divides 1024");
    uint32_t tw[kFillIters];
    u32x4 n0[kFillIters], n1[kFillIters];
#pragma unroll
    for (int f = 0; f < kFillIters; ++f) {
        const uint32_t t = threadIdx.x + f * TPB;
        if constexpr ((LAB & kLabNoTabLoad) != 0) {
            tw[f] = t * 0x9E3779B9u;
            n0[f] = u32x4{t, t ^ 1u, t ^ 2u, t ^ 3u};
            n1[f] = n0[f];
            continue;
        }
        tw[f] = g_tab[t];
        if constexpr (kHalfFold) {
            const uint32_t fk = 2 * (t >> 8) + ((t >> 3) & 1), fe = (t >> 4) & 15, fc = 4 * (t & 7);
            n0[f] = *reinterpret_cast<const u32x4 *>(g_nib + (fk * 16 + fe) * 64 + fc);
        } else {
            n0[f] = *reinterpret_cast<const u32x4 *>(g_nib + 8 * t);
            n1[f] = *reinterpret_cast<const u32x4 *>(g_nib + 8 * t + 4);
        }
    }
    WView cv0 = walk.view(0), cv1 = walk.view(1);
    __builtin_amdgcn_sched_barrier(0);
    Round a0, a1, b0, b1;
    load_round_buf<true>(a0, cv0.p, lane_off, cv0.nb);
    load_round_buf<true>(a1, cv1.p, lane_off, cv1.nb);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < kFillIters; ++f) {
        const uint32_t tt = threadIdx.x + f * TPB, slice = tt >> 8, entry = tt & 255;
        const uint32_t slot0 = ((slice >> 1) << 16 | entry << 8 | (slice & 1) << 7) / 16;
        const uint32_t w = tw[f];
        // 32 copies as 8 x b128, permuted by thread (slot r ^ (tt & 7)) so 8 neighbouring threads hit
        // 8 bank groups; the xor form costs one VALU per store
        const uint32_t byte_t = (slot0 | (tt & 7)) << 4;
#pragma unroll
        for (int r = 0; r < ((LAB & kLabNoFill) ? 0 : 8); ++r)
            *reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(lds) + (byte_t ^ uint32_t(16 * r))) = u32x4{w, w, w, w};
        if constexpr (kHalfFold) {
            reinterpret_cast<u32x4 *>(lds + kHalfFoldOff / 4)[tt] = n0[f];
        } else {
            u32x4 *dst = reinterpret_cast<u32x4 *>(reinterpret_cast<uint8_t *>(lds) + kFoldLdsOff) + 2 * tt;
            dst[0] = n0[f];
            dst[1] = n1[f];
        }
    }
    lds_barrier();
    if constexpr ((LAB & kLabMid) != 0) lab_mid[0] = __builtin_amdgcn_s_memrealtime();
    const Lut t(lds);
    const NibFold nf(lds);
    auto fold = [&](uint32_t x) -> uint32_t {
        if constexpr (kHalfFold) return fold_half(reinterpret_cast<const uint8_t *>(lds), x);
        return nf.apply(x);
    };
    const uint32_t woff = 4 * (lane / G);  // this lane's chunk word within a round
    const uint32_t coff = (lane / G) * BPC;  // its chunk's first byte: the chunk is whole when coff < nb
    WView pv0 = walk.view(2), pv1 = walk.view(3);

    // The stored words through a buffer resource on the round's (wave-uniform) word base: the lane's
    // offset is the only VGPR operand. A 64-bit VGPR address temporary may be allocated on registers
    // of a round still in flight, and the waitcnt pass then drains every load at the loop head.
    // Its range is the round's whole chunks: a partial round's stores past them are dropped.
    auto wrsrc = [](const WView &v) {
        return __builtin_amdgcn_make_buffer_rsrc(v.w, 0, __builtin_amdgcn_readfirstlane(v.nb / (BPC / 4)), 0x00020000);
    };
    auto want_of = [&](const WView &v) -> uint32_t {
        if constexpr (VERIFY) return __builtin_amdgcn_raw_buffer_load_b32(wrsrc(v), woff, 0, 0);
        return 0;
    };
    constexpr bool kHold = HOLD && !VERIFY && G == 8;
    constexpr bool kAddr = !Walk::kLaneView;
    // kHold: lane 8r + c collects chunk c of round r of the current octet (8 rounds) in `line`; up to
    // 8 closed octets wait in hold[] (hold[i] = octet hold_base + nheld - 1 - i) and go out in one
    // burst. With a lane view their addresses come from the walk at flush time (one VGPR per held
    // octet); otherwise each lane keeps its word's address beside it (a segment walk's rounds may
    // belong to different segments).
    // a held word's store. Round 4 measured these as system-scope nt stores too (the staged words'
    // policy): 1 GiB compute 160.6 -> 175.0 us at bpc 512 and 159.5 -> 182.6 at 4096
    // (profiles/r04/r4h_cmp_1g*): write-through 4-byte and 32-byte pieces cost what whole staged
    // lines do not, so they stay plain
    auto held_store = [&](gu8 *p, uint32_t v) { *(gu32 *)p = v; };
    uint32_t line = 0;
    uint32_t hold[kHold ? 8 : 1];
    gu32 *laddr = nullptr;
    gu32 *hold_addr[kHold && kAddr ? 8 : 1];
    uint32_t nheld = 0, hold_base = 0;
    auto flush = [&]() {
#pragma unroll
        for (int i = 0; i < (kHold ? 8 : 0); ++i) {
            // kLabNoStore keeps the words live through a compare that practically never stores
            if (uint32_t(i) < nheld && ((LAB & kLabNoStore) == 0 || hold[i] == 0x9E3779B9u)) {
                if constexpr ((LAB & kLabNearStore) != 0 && !kAddr) {
                    *(gu32 *)((gu8 *)walk.view(0).w + 4 * lane) = hold[i];
                } else if constexpr (kAddr) {
                    if (hold_addr[i]) *hold_addr[i] = hold[i];
                } else {
                    const uint32_t kk = 8 * (hold_base + nheld - 1 - i) + (lane >> 3);
                    if (kk < K) {
                        const WView v = walk.view(kk);
                        if ((lane & 7) * BPC < v.nb) held_store((gu8 *)v.w + 4 * (lane & 7), hold[i]);
                    }
                }
            }
        }
        hold_base += nheld;
        nheld = 0;
    };
    // y: the chunk's finished CRC, byte-swapped (the affine fold image carries init and final xor
    // and the swap: y is the stored big-endian word as it loads)
    // kStageWords (compute at bpc <= 2048 over a contiguous block): every word of a window of
    // kStageMaxRounds rounds per wave waits in the LDS the half fold image leaves free (16 KiB: slot s's round k at
    // word (k * 16 + s) * CPW + c, CPW = 4096 / bpc words per round) and the workgroup writes them at its
    // end as whole runs of 16 * CPW words, since the 16 waves' k-th rounds are 16 consecutive units.
    // The held stores send each wave's words as 32-B pieces of lines that three other waves complete
    // later, into a saturated read stream: 0.4 us of the 1.1 us those writes cost an overlapped 128 MiB
    // launch (profiles/r03/reentry/r3zb_c128_*).
    constexpr bool kStage = !VERIFY && (LAB & kStageWords) != 0 && Walk::kContiguous && kHalfFold && TPB == 1024;
    constexpr uint32_t kCpw = 64 / G;  // chunk words per round
    constexpr uint32_t kSR = kStageMaxRounds(BPC);  // rounds per staging window
    uint32_t *stage = lds + kLdsBytesWave / 4 - 4096;
    const uint32_t slot = threadIdx.x >> 6;
    // Past kSR rounds per wave (bpc 1024 / 2048; bpc 512 with kLabStageWin) a window is written out
    // after the step that finishes round m * kSR - 1, for every m with m * kSR < kq (or m * kSR == kq when
    // some waves have kq + 1 rounds): every wave of the launch has at least kq rounds, so every wave runs
    // that step and meets both barriers. The last window goes out at the workgroup's end.
    // A staged word's store (round 4): system scope (sc0 sc1, written through the L2) and non-temporal
    // (nt), through a buffer resource on the wave-uniform word base with the lane's byte offset as the
    // only VGPR operand. The words then leave no dirty lines for the end-of-kernel release to write
    // back. 128 MiB per launch, lab A/B against plain stores (lab 128) over two boxes: overlapped
    // -0.64 / -0.29 us, barriered -0.86 us (profiles/r04/r4e_cmp_*, r4f_cmp_*); system scope alone
    // -0.16 / -0.44 and -0.26, nt alone -0.22 / -0.21 and -0.14. The buffer offset is 31-bit:
    // launch_wave3 stages only launches whose words stay below 2 GiB (data below 256 GiB at bpc 512).
    auto stage_store = [&](gu8 *p, uint32_t v) {
        // kLabNoStore (diagnostic 118): the staged words are kept live (a store that practically never
        // happens) but not written: what the flush's global stores cost a launch (wrong results)
        if constexpr ((LAB & kLabNoStore) != 0) {
            if (v != 0x9E3779B9u) return;
        }
        if constexpr (kStage && (LAB & kLabStorePlain) == 0) {
            const uint64_t wb = rfl64(reinterpret_cast<uint64_t>(walk.words));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<void *>(wb), 0, 0x7FFFFFFF, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(v, rs, uint32_t(reinterpret_cast<uint64_t>(p) - wb), 0, 1 | 2 | 16);
        } else {
            *(gu32 *)p = v;
        }
    };
    uint32_t kq_flush = 0;  // flush at kend <= kq_flush
    if constexpr (kStage) kq_flush = walk.kq - (walk.kr == 0 ? 1u : 0u);
    auto stage_flush = [&](uint32_t kend) {
        if constexpr (kStage) {
            if (kend % kSR == 0 && kend <= kq_flush && walk.kq != 0) {
                lds_barrier();
                const uint64_t wg_first = walk.first - slot;
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const uint32_t t = threadIdx.x + 1024 * p, kk = t / (16 * kCpw), s = (t / kCpw) & 15,
                                   c = t % kCpw;
                    stage_store((gu8 *)walk.words +
                                    4 * kCpw * (wg_first + s + uint64_t(kend - kSR + kk) * walk.stride) + 4 * c,
                                stage[t]);
                }
                lds_barrier();
            }
        }
    };
    // compute at bpc 4096 (one word per round) over one contiguous block: lane k % 64 keeps round k's
    // word, and one store per 64 rounds writes them, instead of a 4-byte store per round into the read
    // stream: 128 MiB 23.63 -> 22.54 us overlapped, 25.24 -> 24.51 barriered, 1 GiB 160.6 -> 158.8
    // (verify 157.7; profiles/r03/reentry/r3zq_*)
    constexpr bool kHold64 = !VERIFY && G == 64 && Walk::kContiguous && (LAB & kLabNoHold) == 0;
    uint32_t line64 = 0;
    auto finish = [&](uint32_t k, const WView &v, uint32_t y, uint32_t want) {
        if constexpr (kHold64) {
            // lane 0 holds the chunk's word (group_xor)
            if (k >= K) return;
            const uint32_t yy = __builtin_amdgcn_readfirstlane(y);
            line64 = lane == (k & 63) ? yy : line64;
            if ((k & 63) == 63 || k + 1 == K) {
                const uint32_t kk = (k & ~63u) + lane;
                if (lane <= (k & 63)) held_store((gu8 *)walk.view(kk).w, line64);
            }
            return;
        }
        if constexpr (kStage) {
            if (k < K && j == 0) stage[((k % kSR) * 16 + slot) * kCpw + lane / G] = y;
            return;
        }
        if constexpr (kHold) {
            if (k >= K) return;
            const uint32_t r = k & 7;
            // group c's lanes all hold chunk c's state (group_xor is a butterfly)
            const uint32_t got = uint32_t(__builtin_amdgcn_ds_bpermute(int(32 * (lane & 7)), int(y)));
            const bool mine = (lane >> 3) == r;
            line = mine ? got : line;
            if constexpr (kAddr)
                laddr = mine ? ((lane & 7) * BPC < v.nb ? (gu32 *)((gu8 *)v.w + 4 * (lane & 7)) : nullptr) : laddr;
            if (r == 7 || k + 1 == K) {
#pragma unroll
                for (int i = (kHold ? 7 : 0); i > 0; --i) {
                    hold[i] = hold[i - 1];
                    if constexpr (kAddr) hold_addr[i] = hold_addr[i - 1];
                }
                hold[0] = line;
                if constexpr (kAddr) {
                    hold_addr[0] = laddr;
                    laddr = nullptr;
                }
                if (++nheld == 8) flush();
            }
            return;
        }
        if (k >= K || j != 0) return;
        const uint32_t c = y;
        if constexpr (VERIFY) {
            // the diagnostics compute wrong CRCs: compare inverted so they do not flag every chunk
            // (an atomic per chunk would dominate their time); a partial round's lanes past its
            // whole chunks computed zeros
            if ((want != c) != kWrong && coff < v.nb)
                __hip_atomic_fetch_max((gu64 *)result, ~(unsigned long long)(v.key + lane / G), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(c, wrsrc(v), woff, 0, 0);
        }
    };
    auto word = [](const Round &r, int i) -> uint32_t { return r.w[i >> 2][i & 3]; };
    // the table step of one word (kLabNoMath, diagnostic: a plain XOR instead, wrong on purpose)
    auto look = [&](uint32_t x) -> Look {
        if constexpr (NOMATH) return Look{{x, 0u, 0u, 0u}};
        return lookups(t, x);
    };
    // two interleaved chains over c0, c1 (chain 1's 4 reads fly while chain 0 folds). A chain ends in
    // x = state ^ w15, before the last word's table step: the lane fold's image carries that step
    // (build_fold_nibbles_pre), 60 lookups per lane and round instead of 64
    auto chains = [&](Round &c0, Round &c1, uint32_t &x0, uint32_t &x1) {
        x0 = word(c0, 0);
        x1 = word(c1, 0);
        Look l0 = look(x0), l1;
        __builtin_amdgcn_sched_barrier(0);
        if constexpr ((LAB & kLabFull16) != 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                l1 = look(x1);
                __builtin_amdgcn_sched_barrier(0);
                x0 = combine(l0, i < 15 ? word(c0, i < 15 ? i + 1 : 15) : 0u);
                __builtin_amdgcn_sched_barrier(0);
                if (i < 15) l0 = look(x0);
                __builtin_amdgcn_sched_barrier(0);
                x1 = combine(l1, i < 15 ? word(c1, i < 15 ? i + 1 : 15) : 0u);
                __builtin_amdgcn_sched_barrier(0);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 15; ++i) {
            l1 = look(x1);
            __builtin_amdgcn_sched_barrier(0);
            x0 = combine(l0, word(c0, i + 1));
            __builtin_amdgcn_sched_barrier(0);
            if (i < 14) l0 = look(x0);
            __builtin_amdgcn_sched_barrier(0);
            x1 = combine(l1, word(c1, i + 1));
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // one round as a single chain. The two solo rounds of the last step end in different asm markers:
    // identical code otherwise gets tail-merged into one copy that both run (register copies in).
    auto solo = [&](Round &c, const WView &v, uint32_t k, uint32_t w, auto id) {
        uint32_t x = word(c, 0);
        if constexpr ((LAB & kLabFull16) != 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x = combine(look(x), i < 15 ? word(c, i < 15 ? i + 1 : 15) : 0u);
        } else {
#pragma unroll
            for (int i = 0; i < 15; ++i) x = combine(look(x), word(c, i + 1));
        }
        finish(k, v, group_xor<G>(fold(x)), w);
        if constexpr (decltype(id)::value == 0) asm volatile("; solo round 0" ::: "memory");
        else asm volatile("; solo round 1" ::: "memory");
    };
    // A step: the words of rounds k, k+1 are requested first (older than the prefetch, so waiting for
    // them never drains it: vmcnt is in-order), then the prefetch of rounds k+2, k+3 into p0, p1 (past
    // the wave's last round: the cache-resident table image), then the chains over c0, c1. The next
    // views are resolved at the end.
    // LATE (production): the prefetch goes out once this step's rounds have landed, so at most 8 KiB
    // are in flight per wave (128 KiB per CU), not 16: more requests in flight lower the DRAM
    // efficiency (docs/DESIGN_HISTORY.md §5.0). kLabEarly (lab A/B): issued at the start of the step.
    // priority by rounds left (kPrioMinRounds); wave-uniform, so the branches are SALU
    const bool use_prio = (LAB & kLabPrio) != 0 || ((LAB & kLabNoPrio) == 0 && K >= kPrioMinRounds);
    auto prio = [&](uint32_t k) {
        if (use_prio) {
            const uint32_t left = K > k ? K - k : 0;
            if (left * 4 > 3 * K) __builtin_amdgcn_s_setprio(3);
            else if (left * 4 > 2 * K) __builtin_amdgcn_s_setprio(2);
            else if (left * 4 > K) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
    };
    auto step = [&](Round &c0, Round &c1, Round &p0, Round &p1, uint32_t k) {
        prio(k);
        const uint32_t w0 = want_of(cv0), w1 = want_of(cv1);
        if constexpr (!LATE) {
            load_round_buf<true>(p0, pv0.p, lane_off, pv0.nb);
            load_round_buf<true>(p1, pv1.p, lane_off, pv1.nb);
        }
        __builtin_amdgcn_sched_barrier(0);
        regroup(c0);
        regroup(c1);
        if constexpr ((LAB & kLabMid) != 0) {
            if (k == 0) lab_mid[1] = __builtin_amdgcn_s_memrealtime();  // the first rounds' data landed
        }
        if constexpr (LATE) {
            __builtin_amdgcn_sched_barrier(0);
            load_round_buf<true>(p0, pv0.p, lane_off, pv0.nb);
            load_round_buf<true>(p1, pv1.p, lane_off, pv1.nb);
            __builtin_amdgcn_sched_barrier(0);
        }
        uint32_t x0, x1;
        chains(c0, c1, x0, x1);
        finish(k, cv0, group_xor<G>(fold(x0)), w0);
        finish(k + 1, cv1, group_xor<G>(fold(x1)), w1);
        stage_flush(k + 2);
        __builtin_amdgcn_sched_barrier(0);
        cv0 = pv0;
        cv1 = pv1;
        pv0 = walk.view(k + 4);
        pv1 = walk.view(k + 5);
    };

    // The A -> B -> A rotation by unrolling. Every loop has one exit, at its bottom, and every step
    // in it is the same code: an exit from the middle of the body, or a special last step that values
    // reach from both buffer sets, makes the register allocator copy the rounds (32 v_mov per step).
    const uint32_t nr = (K + 1) & ~1u;  // rounds rounded up to whole steps
    if constexpr (SOLO) {
        // The last step outside the loop, its two rounds as single chains one after the other: the
        // first chain overlaps the second round's arrival, and only one round's lookups remain once
        // the wave's last data has landed. Its buffers are STATIC: with F = nr / 2 - 1 full steps,
        // F even runs pairs A -> B -> A and ends in A; F odd runs one step A -> B, then pairs
        // B -> A -> B, and ends in B. Two copies of the loop; no value crosses between them.
        auto last = [&](Round &c0, Round &c1, uint32_t k) {
            prio(k);
            const uint32_t w0 = want_of(cv0), w1 = want_of(cv1);
            __builtin_amdgcn_sched_barrier(0);
            regroup(c0);
            solo(c0, cv0, k, w0, std::integral_constant<int, 0>{});
            regroup(c1);
            solo(c1, cv1, k + 1, w1, std::integral_constant<int, 1>{});
            stage_flush(k + 2);
        };
        if (nr != 0) {
            const uint32_t kl = nr - 2;  // the last step's first round
            if ((kl >> 1) & 1) {
                step(a0, a1, b0, b1, 0);
                for (uint32_t k = 2; k < kl; k += 4) {
                    step(b0, b1, a0, a1, k);
                    step(a0, a1, b0, b1, k + 2);
                }
                last(b0, b1, kl);
            } else {
                for (uint32_t k = 0; k < kl; k += 4) {
                    step(a0, a1, b0, b1, k);
                    step(b0, b1, a0, a1, k + 2);
                }
                last(a0, a1, kl);
            }
        }
    } else {
        for (uint32_t k = 0; k < nr; k += 4) {
            step(a0, a1, b0, b1, k);
            if (k + 2 >= nr) break;
            step(b0, b1, a0, a1, k + 2);
        }
    }
    if constexpr (kStage) {
        lds_barrier();  // every wave of the workgroup runs wave_rounds to its end
        const uint64_t wg_first = walk.first - slot;
        const uint32_t wb = walk.kq ? kSR * (kq_flush / kSR) : 0u;  // the last window's first round
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t t = threadIdx.x + 1024 * p, k = wb + t / (16 * kCpw), s = (t / kCpw) & 15, c = t % kCpw;
            const uint32_t ks = walk.kq + (wg_first + s < walk.kr ? 1u : 0u);
            if (k < ks)
                stage_store((gu8 *)walk.words + 4 * (kRoundBytes / BPC) * (wg_first + s + uint64_t(k) * walk.stride) +
                                4 * c,
                            stage[t]);
        }
    } else if constexpr (kHold) {
        flush();
    }
}

// Slow region of one contiguous run: the chunks after its last whole round plus its short tail, one
// chunk per thread of the grid (at most 8 + 1), 128-byte lines (crc_run_lines).
template <int BPC, bool VERIFY, int TPB = kBlockThreads>
__device__ __forceinline__ void slow_region(const uint32_t *lds, const uint8_t *sdata, uint8_t *sw, uint64_t len,
                                            uint64_t skey, int check_short_tail, unsigned long long *result) {
    constexpr int kChunksPerUnit = kRoundBytes / BPC;
    const Lut t(lds);
    const uint64_t nfull = len / BPC;
    const uint64_t first_slow = (len / kRoundBytes) * kChunksPerUnit;
    const uint64_t nslow = nfull - first_slow + (len % BPC ? 1 : 0);
    const uint64_t gtid = uint64_t(blockIdx.x) * TPB + threadIdx.x;
    const bool crc_al4 = (reinterpret_cast<uintptr_t>(sw) & 3u) == 0;
    if (gtid < nslow) {
        const uint64_t chunk = first_slow + gtid;
        const uint32_t sz = chunk < nfull ? uint32_t(BPC) : uint32_t(len % BPC);
        const uint32_t c = ~crc_run_lines(t, 0xFFFFFFFFu, sdata + chunk * BPC, sz);
        if constexpr (VERIFY) {
            if ((sz == uint32_t(BPC) || check_short_tail) && load_be32(sw + 4 * chunk, crc_al4) != c)
                atomicMax(result, ~(unsigned long long)(skey + chunk));
        } else {
            store_be32(sw + 4 * chunk, c, crc_al4);
        }
    }
}

// The short last chunk (len % BPC bytes) of a run whose whole chunks the walk covered: one lane
// of workgroup 0.
template <int BPC, bool VERIFY, int TPB = kBlockThreads>
__device__ __forceinline__ void short_tail(const uint32_t *lds, const uint8_t *sdata, uint8_t *sw, uint64_t len,
                                           uint64_t skey, int check_short_tail, unsigned long long *result) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const Lut t(lds);
    const uint64_t chunk = len / BPC;
    const bool crc_al4 = (reinterpret_cast<uintptr_t>(sw) & 3u) == 0;
    const uint32_t c = ~crc_run_lines(t, 0xFFFFFFFFu, sdata + chunk * BPC, uint32_t(len % BPC));
    if constexpr (VERIFY) {
        if (check_short_tail && load_be32(sw + 4 * chunk, crc_al4) != c)
            atomicMax(result, ~(unsigned long long)(skey + chunk));
    } else {
        store_be32(sw + 4 * chunk, c, crc_al4);
    }
}

// One block (PITCH = false) or a constant-pitch stream (PITCH = true, ChunkLaunch::pitch/npk/geom).
template <int BPC, bool VERIFY, bool PITCH, bool SOLO, int LAB = 0, int TPB = kBlockThreads>
__global__ __launch_bounds__(TPB) void crc32c_wave_kernel(ChunkLaunch a, const uint32_t *__restrict__ g_tab,
                                                                    const uint32_t *__restrict__ g_nib) {
    static_assert(BPC <= kRoundBytes && BPC % 512 == 0, "one-round units");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytesWave / 4];
    constexpr int kCpu = kRoundBytes / BPC;
    constexpr int kWpb = TPB / 64;
    const uint64_t nwaves = uint64_t(gridDim.x) * kWpb;
    const uint64_t wave = uint64_t(blockIdx.x) * kWpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *words = VERIFY ? const_cast<uint8_t *>(a.crc_be) : a.out_be;
    const uint8_t *dummy = reinterpret_cast<const uint8_t *>(g_tab);
    constexpr bool kHold = !VERIFY && BPC == 512 && (LAB & kLabNoHold) == 0;
    // the wave's round count from the host's split (ChunkLaunch::kq/kr): SALU only
    const uint32_t K = a.kq + (wave < a.kr ? 1u : 0u);
    unsigned long long lab_mid[3] = {0, 0, 0};  // kLabMid only
#if HDFS3_LAB
    LabClock clk;
    if constexpr ((LAB & kLabClock) != 0) clk.start();
    if constexpr ((LAB & kLabMid) != 0) {
        asm volatile("" ::"s"(a.kq), "s"(a.kr));  // the kernel arguments have landed
        lab_mid[2] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if constexpr (PITCH) {
        const PacketGeom &g = a.geom;
        PitchWalk<kCpu> w{a.data, words, a.pitch, a.crc_pitch ? a.crc_pitch : a.pitch, wave, nwaves, K,
                          g.upp, g.magic, g.shift, g.ptail, g.lunits, g.ltail, uint32_t(a.npk - 1), dummy};
        wave_rounds<BPC, VERIFY, SOLO, kHold, LAB, TPB>(w, lds, g_tab, g_nib, a.result);
        const uint64_t lp = a.npk - 1;
        if (a.last_len % BPC)  // wave-uniform: only the last packet's short chunk is left
            short_tail<BPC, VERIFY, TPB>(lds, a.data + lp * a.pitch, words + lp * w.wpitch, a.last_len, lp << 32,
                                         a.check_short_tail, a.result);
    } else {
        BlockWalk<kCpu> w{a.data, words, a.chunk_base, wave, nwaves, K, dummy, a.kq, a.kr};
        wave_rounds<BPC, VERIFY, SOLO, kHold, LAB, TPB>(w, lds, g_tab, g_nib, a.result, lab_mid);
        if (a.len % kRoundBytes)  // wave-uniform: a block of whole rounds has no slow region
            slow_region<BPC, VERIFY, TPB>(lds, a.data, words, a.len, a.chunk_base, a.check_short_tail, a.result);
    }
#if HDFS3_LAB
    if constexpr ((LAB & kLabClock) != 0) {
        if constexpr ((LAB & kLabMid) != 0)
            clk.end(a.lab_seq, ((lab_mid[0] - clk.r0) & 0x1FFFFF) | ((lab_mid[1] - clk.r0) & 0x1FFFFF) << 21 |
                                   ((lab_mid[2] - clk.r0) & 0x1FFFFF) << 42);
        else
            clk.end(a.lab_seq);
    }
#endif
}

// A list of segments (blocks of a batch, packets of a descriptor list): the core over a SegWalk
// (a segment's last unit partial when its whole chunks end inside a round), then every segment's
// short last chunk, one lane each.
template <int BPC, bool VERIFY, bool UNI, int LAB = 0, int TPB = kBlockThreads>
__global__ __launch_bounds__(TPB) void crc32c_segments_kernel(SegLaunch L, const uint32_t *__restrict__ g_tab,
                                                              const uint32_t *__restrict__ g_nib) {
    static_assert(BPC <= kRoundBytes && BPC % 512 == 0, "one-round units");
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytesWave / 4];
    constexpr int kCpu = kRoundBytes / BPC;
    constexpr int kWpb = TPB / 64;
    const uint64_t nwaves = uint64_t(gridDim.x) * kWpb;
    const uint64_t wave = uint64_t(blockIdx.x) * kWpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    SegWalk<kCpu, UNI> w{(CSegLaunch *)(&L), wave, nwaves, L.kq + (wave < L.kr ? 1u : 0u),
                         reinterpret_cast<const uint8_t *>(g_tab)};
    wave_rounds<BPC, VERIFY, false, !VERIFY && BPC == 512, LAB, TPB>(w, lds, g_tab, g_nib, L.result);

    // every whole chunk was in a (possibly partial) round: only the segments' short last chunks
    // are left, one lane each, item i on workgroup i % grid (piece CRCs for a combine: the caller's)
    if (L.dense_words) return;
    const Lut t(lds);
    for (uint64_t si = uint64_t(threadIdx.x) * gridDim.x + blockIdx.x; si < L.nseg;
         si += uint64_t(gridDim.x) * TPB) {
        DevSegment sd;
        if (L.stride) {
            sd = L.inl[0];
            sd.data += si * L.stride;
            sd.crc += si * L.stride;
            sd.len = si + 1 < L.nseg ? L.inl[0].len : L.inl[1].len;
            sd.key_base = si << 32;
        } else {
            sd = L.seg ? L.seg[si] : L.inl[si];  // per-thread index: vector loads
        }
        if (sd.len % BPC) {
            const uint64_t c = sd.len / BPC;
            const uint32_t v = ~crc_run_lines(t, 0xFFFFFFFFu, sd.data + c * BPC, uint32_t(sd.len % BPC));
            if constexpr (VERIFY) {
                if (L.check_short_tail && load_be32(sd.crc + 4 * c, true) != v)
                    atomicMax(L.result, ~(unsigned long long)(sd.key_base + c));
            } else {
                store_be32(sd.crc + 4 * c, v, true);
            }
        }
    }
}

// Overlapped launches up to 256 MiB end with the solo last step. Verify, 128 MiB at bpc 512:
// 21.52 -> 20.71 us per launch against the interleaved last step (variant 93), 21.45 -> 21.02
// against the round-2 kernel (profiles/r03/r3h_ab_ovl.jsonl, r3g_ab_ovl.jsonl); compute at bpc
// 512: 22.63 -> 22.24 us (variant 94 before it became production, r3i_ab_cmp_ovl.jsonl).
// Barriered launches and launches past 256 MiB keep the interleaved last step (round 2: +0.9 us
// barriered and +1 % at 1 GiB with it).
constexpr uint64_t kSoloTailMaxBytes = uint64_t(256) << 20;

// SOLO: the solo last step when the launch qualifies (above); LAB: lab A/B bits.
template <int BPC, bool V, bool PITCH, bool SOLO, int LAB = 0, int TPB = kBlockThreads>
hipError_t launch_wave3(const ChunkLaunch &a, const uint32_t *tab, const uint32_t *fold, int grid_cap, hipStream_t s) {
    constexpr int G = BPC / 64;
    constexpr int set = G == 8 ? 0 : G == 16 ? 1 : G == 32 ? 2 : 3;
    const uint32_t *nib = fold + ((LAB & kLabFull16) ? kFoldAffineOldOff : kFoldAffineOff) + set * kFoldNibbleWords;
    const uint64_t units = PITCH ? (a.npk - 1) * a.geom.upp + a.geom.lunits : a.len / kRoundBytes;
    const uint64_t rpw = (LAB & kLabOneRound) != 0 && units <= 4096 ? 1 : 2;  // rounds per wave planned
    const uint64_t need = (units + rpw * (TPB / 64) - 1) / (rpw * (TPB / 64));
    int grid = int(need < uint64_t(grid_cap) ? need : uint64_t(grid_cap));
    if (grid < 1) grid = 1;
    // units over the grid's waves: wave w takes kq rounds, plus one when w < kr (32-bit round counts:
    // 16 TiB per launch; ChunkLaunch::kq/kr)
    const uint64_t nwaves = uint64_t(grid) * (TPB / 64);
    if (units / nwaves >= (uint64_t(1) << 32)) return hipErrorInvalidValue;
    ChunkLaunch b = a;
    if constexpr ((LAB & kLabClock) != 0) b.lab_seq = g_lab_seq++;
    b.kq = uint32_t(units / nwaves);
    b.kr = uint32_t(units % nwaves);
    // Verify launches below 64 MiB take smaller workgroups (round 4): a 1024-thread workgroup fills a
    // CU's LDS, so with 2 rounds per wave a launch of fewer than 8,192 rounds (32 MiB) left CUs idle and
    // every CU it used paid the whole table fill for few rounds. 256 threads up to 16 MiB, 512 up to
    // 64 MiB, HBM-resident blocks, wall clock per launch (tools/ab.py, profiles/r04/r4h_*): 4 MiB
    // 7.38 -> 6.45 us barriered, 7.05 -> 6.43 overlapped; 16 MiB 7.95 -> 6.47 / 7.27 -> 5.81; 32 MiB
    // 10.16 -> 9.04 / 8.82 -> 8.53; 64 MiB 14.57 -> 13.90 / 13.36 -> 12.56; the block reader's
    // 64-packet batch (4 MiB, cache-resident) 7.00 -> 4.43. 128 MiB stays at 1024 (256 / 512 threads:
    // +6.1 / +0.4 us barriered). Compute over a contiguous block keeps 1024 threads: its staged words
    // need the whole LDS; compute over a packet stream (the writer's batches: held stores) does not.
    if constexpr ((V || PITCH) && TPB == 1024 && (LAB & kLabWg1024) == 0) {
        // compute over a packet stream of <= 16 MiB (the writer's batches): each round's words stored at
        // once. With two rounds per wave the held stores only delay the words to the wave's end: the
        // writer's 64-packet batch 5.32 -> 4.47 us against 4.41 for its verify (lab 163, round 6,
        // profiles/r06/r6n_partial_rate.jsonl)
        constexpr int kSmall = (!V && PITCH) ? kLabNoHold : 0;
        if (units <= 4096) return launch_wave3<BPC, V, PITCH, SOLO, LAB | kSmall, 256>(a, tab, fold, grid_cap, s);
        if (units <= 16384) return launch_wave3<BPC, V, PITCH, SOLO, LAB, 512>(a, tab, fold, grid_cap, s);
    }
    // compute at bpc <= 2048 over one contiguous block: staged words; at bpc 512 only while they fit one
    // window (beyond it the held stores measured faster at 1 GiB: 160.4 against 163.1 us in windows)
    if constexpr (!V && BPC <= 2048 && !PITCH && TPB == 1024 &&
                  (LAB & (kStageWords | kLabNoStage | kLabNoHold)) == 0) {
        const bool words_fit = units * uint64_t(4 * (kRoundBytes / BPC)) < (uint64_t(1) << 31);  // stage_store
        if (words_fit && (b.kq + (b.kr ? 1u : 0u) <= kStageMaxRounds(BPC) || BPC != 512 || (LAB & kLabStageWin) != 0))
            return launch_wave3<BPC, V, PITCH, SOLO, LAB | kStageWords, TPB>(a, tab, fold, grid_cap, s);
    }
    if (a.overlap_previous) {  // AQL packet without the barrier bit (HDFS3_LAUNCH_OVERLAP_PREVIOUS)
        if constexpr (SOLO) {
            if (units * kRoundBytes <= kSoloTailMaxBytes) {
                hipExtLaunchKernelGGL((crc32c_wave_kernel<BPC, V, PITCH, true, LAB, TPB>), dim3(grid),
                                      dim3(TPB), 0, s, nullptr, nullptr, hipExtAnyOrderLaunch, b, tab, nib);
                return hipGetLastError();
            }
        }
        hipExtLaunchKernelGGL((crc32c_wave_kernel<BPC, V, PITCH, false, LAB, TPB>), dim3(grid),
                              dim3(TPB), 0, s, nullptr, nullptr, hipExtAnyOrderLaunch, b, tab, nib);
    } else {
        hipLaunchKernelGGL((crc32c_wave_kernel<BPC, V, PITCH, false, LAB, TPB>), dim3(grid), dim3(TPB),
                           0, s, b, tab, nib);
    }
    return hipGetLastError();
}

// The grid and the waves' round split (SegLaunch::kq/kr) are set here. Small launches take
// smaller workgroups, as launch_wave3's verifies do (round 6): a 1024-thread workgroup owns a CU's
// LDS, so a 64-packet batch (1,024 units) ran on 32 CUs.
template <int BPC, bool V, int LAB = 0, int TPB = kBlockThreads>
hipError_t launch_segments3(const SegLaunch &in, const uint32_t *tab, const uint32_t *fold, int grid_cap,
                            hipStream_t s) {
    if constexpr (TPB == 1024) {
        if (in.units <= 4096) return launch_segments3<BPC, V, LAB, 256>(in, tab, fold, grid_cap, s);
        if (in.units <= 16384) return launch_segments3<BPC, V, LAB, 512>(in, tab, fold, grid_cap, s);
    }
    constexpr int G = BPC / 64;
    constexpr int set = G == 8 ? 0 : G == 16 ? 1 : G == 32 ? 2 : 3;
    constexpr uint64_t kWpb = TPB / 64;
    const uint32_t *nib = fold + ((LAB & kLabFull16) ? kFoldAffineOldOff : kFoldAffineOff) + set * kFoldNibbleWords;
    SegLaunch L = in;
    const uint64_t need = (L.units + 2 * kWpb - 1) / (2 * kWpb);
    const uint64_t tail_need = (L.nseg + TPB - 1) / TPB;
    uint64_t g = need > tail_need ? need : tail_need;
    g = g < uint64_t(grid_cap) ? g : uint64_t(grid_cap);
    const int grid = int(g > 0 ? g : 1);
    const uint64_t nwaves = uint64_t(grid) * kWpb;
    if (L.units / nwaves >= (uint64_t(1) << 32)) return hipErrorInvalidValue;
    L.kq = uint32_t(L.units / nwaves);
    L.kr = uint32_t(L.units % nwaves);
    if (L.uniform)
        hipLaunchKernelGGL((crc32c_segments_kernel<BPC, V, true, LAB, TPB>), dim3(grid), dim3(TPB), 0, s, L, tab, nib);
    else
        hipLaunchKernelGGL((crc32c_segments_kernel<BPC, V, false, LAB, TPB>), dim3(grid), dim3(TPB), 0, s, L, tab, nib);
    return hipGetLastError();
}

}  // namespace
}  // namespace hdfs3crc
