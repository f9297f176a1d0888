// Slice-by-4 CRC32C tables (reflected poly 0x82F63B78), generated at run time.
//
// T[0] is the byte table of SWCrc32c (src/common/SWCrc32c.cpp:47-91, used at :102):
//   crc = T[0][(crc ^ b) & 0xFF] ^ (crc >> 8).
// T[k][b] = T[0][T[k-1][b] & 0xFF] ^ (T[k-1][b] >> 8) advances k more zero bytes,
// so one little-endian 32-bit word w is consumed as
//   c ^= w; c = T[3][c & 0xFF] ^ T[2][(c >> 8) & 0xFF] ^ T[1][(c >> 16) & 0xFF] ^ T[0][c >> 24].
#pragma once

#include <cstdint>

namespace hdfs3crc {

constexpr uint32_t kPolyReflected = 0x82F63B78u;  // CRC32C (Castagnoli), CHECKSUM_CRC32C
// CRC-32 (IEEE 802.3 / zlib / boost::crc_32_type, Crc32.h:41-75), CHECKSUM_CRC32: same
// reflected form, init and final xor, so only the tables differ
constexpr uint32_t kPolyCrc32 = 0xEDB88320u;
constexpr int kSlices = 4;
constexpr int kTableEntries = 256;
constexpr int kTableWords = kSlices * kTableEntries;  // 1024 words = 4 KiB image

inline void build_slice_tables(uint32_t out[kSlices][kTableEntries], uint32_t poly = kPolyReflected) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? poly : 0u);
        out[0][i] = c;
    }
    for (int k = 1; k < kSlices; ++k)
        for (int i = 0; i < 256; ++i)
            out[k][i] = out[0][out[k - 1][i] & 0xFFu] ^ (out[k - 1][i] >> 8);
}

// GF(2)-linear "advance the raw CRC state over n zero bytes" as a 32x32 bit matrix
// stored by columns: shift(x) = XOR of cols[i] over the set bits i of x. Used to fold
// partial CRCs of consecutive segments: crc(A||B) = shift_|B|(crc(A)) ^ crc0(B).
inline uint32_t advance_bytes(const uint32_t t0[kTableEntries], uint32_t s, uint64_t n) {
    while (n--) s = t0[s & 0xFFu] ^ (s >> 8);
    return s;
}

inline uint32_t apply_cols(const uint32_t cols[32], uint32_t x) {
    uint32_t y = 0;
    for (int i = 0; i < 32; ++i)
        if ((x >> i) & 1u) y ^= cols[i];
    return y;
}

inline void shift_cols(const uint32_t t0[kTableEntries], uint64_t n, uint32_t cols[32]) {
    for (int i = 0; i < 32; ++i) cols[i] = advance_bytes(t0, 1u << i, n);
}

// Lane-fold matrices for the round kernel: for G lanes per chunk (64-byte segments),
// lane j's partial state is advanced over (G-1-j)*64 bytes. Sets for G = 8,16,32,64
// are packed at word offsets kFoldOffset[g]*32; the 4096-byte advance (round-to-round
// combine for bpc > 4096) follows at kFoldAdvance4096.
constexpr int kFoldGs[4] = {8, 16, 32, 64};
constexpr int kFoldOffset[4] = {0, 8, 24, 56};
constexpr int kFoldAdvance4096 = 120 * 32;
constexpr int kFoldWords = kFoldAdvance4096 + 32;

inline int fold_set_index(int g) { return g == 8 ? 0 : g == 16 ? 1 : g == 32 ? 2 : 3; }

inline void build_fold_matrices(const uint32_t t0[kTableEntries], uint32_t out[kFoldWords]) {
    uint32_t f64[32];
    shift_cols(t0, 64, f64);
    for (int s = 0; s < 4; ++s) {
        const int g = kFoldGs[s];
        uint32_t m[32];
        for (int i = 0; i < 32; ++i) m[i] = 1u << i;  // identity: lane g-1 needs no advance
        for (int j = g - 1; j >= 0; --j) {
            for (int i = 0; i < 32; ++i) out[(kFoldOffset[s] + j) * 32 + i] = m[i];
            for (int i = 0; i < 32; ++i) m[i] = apply_cols(f64, m[i]);
        }
    }
    shift_cols(t0, 4096, out + kFoldAdvance4096);
}

// Lane-specific fold as LDS nibble tables (the round kernels' fold): for each of the
// 64 lanes of a wave, lane j = lane % G, nibble k (0..7) and value e (0..15), the entry
// M_j(e << 4k). Word index ((k * 16 + e) * 64 + lane): every lane reads its own bank.
constexpr int kFoldNibbleWords = 8 * 16 * 64;  // 32 KiB per G

inline void build_fold_nibbles(const uint32_t fold[kFoldWords], int set, uint32_t out[kFoldNibbleWords]) {
    const int g = kFoldGs[set];
    for (int lane = 0; lane < 64; ++lane) {
        const uint32_t *cols = fold + (kFoldOffset[set] + lane % g) * 32;
        for (int k = 0; k < 8; ++k)
            for (uint32_t e = 0; e < 16; ++e)
                out[(k * 16 + e) * 64 + lane] = apply_cols(cols, e << (4 * k));
    }
}

// The round kernel's sets take a chain's state BEFORE its last word's table step (round 5): lane j's
// 16-word chain ends in x = s ^ w15, whose finished state is T(x) (T = the 4-byte slice-by-4 step,
// linear), so the entry M_j(T(e << 4k)) folds T into the lane fold and the kernel skips the last
// word's 4 lookups (64 -> 60 slice lookups per lane and round).
inline void build_fold_nibbles_pre(const uint32_t t0[kTableEntries], const uint32_t fold[kFoldWords], int set,
                                   uint32_t out[kFoldNibbleWords]) {
    const int g = kFoldGs[set];
    for (int lane = 0; lane < 64; ++lane) {
        const uint32_t *cols = fold + (kFoldOffset[set] + lane % g) * 32;
        for (int k = 0; k < 8; ++k)
            for (uint32_t e = 0; e < 16; ++e)
                out[(k * 16 + e) * 64 + lane] = apply_cols(cols, advance_bytes(t0, e << (4 * k), 4));
    }
}

// Affine lane-fold nibble sets (the production round kernel, crc32c_wave.h): the sets above with
// the chunk's init and final xor folded in. By linearity the CRC of a chunk of C = 64 G bytes is
//   ~state(init ~0) = crc0 ^ A^C(~0) ^ ~0,   crc0 = XOR_j M_j(x_j) over chains started from 0,
// so adding the constant K_C = A^C(~0) ^ ~0 to every k = 0 entry of lane G-1 (whose M is the
// identity) makes the lane fold + group xor return the finished CRC: no init xor per round and
// no final complement per chunk. Every entry is then byte-swapped: the fold is linear in its entries,
// so the group xor returns the CRC already in the big-endian order of the stored words (no v_perm per
// round to compare or store them).
// The device fold image is the kFoldWords matrix columns followed by the 4 affine sets.
constexpr int kFoldAffineOff = kFoldWords;
// (lab A/B, round 5: the round-4 sets on the chain's finished state follow at kFoldAffineOldOff)
constexpr int kFoldAffineOldOff = kFoldAffineOff + 4 * kFoldNibbleWords;
constexpr int kFoldImageWords = kFoldAffineOldOff + 4 * kFoldNibbleWords;
// `out` holds set `set` built by build_fold_nibbles_pre; adds K_C in place
inline void build_fold_affine(const uint32_t t0[kTableEntries], int set, uint32_t out[kFoldNibbleWords]) {
    const int g = kFoldGs[set];
    const uint32_t kc = advance_bytes(t0, 0xFFFFFFFFu, uint64_t(64) * g) ^ 0xFFFFFFFFu;
    for (int lane = 0; lane < 64; ++lane)
        if (lane % g == g - 1)
            for (uint32_t e = 0; e < 16; ++e) out[e * 64 + lane] ^= kc;  // k = 0
    for (int i = 0; i < kFoldNibbleWords; ++i) out[i] = __builtin_bswap32(out[i]);
}

}  // namespace hdfs3crc
