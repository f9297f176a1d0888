// Host check of the round kernel's lane-fold image (crc32c_tables.h), run by tests/test_fold_image.py
// (CPU suite): the round kernel's arithmetic for one 4 KiB round restated on the CPU — lane l holds
// bytes [64 l, 64 l + 64), a chunk of G * 64 bytes is G consecutive lanes, each lane a chain of table
// steps from state 0, then its nibble fold entries and the xor over the chunk's lanes — must give every
// chunk's CRC32C (byte-swapped, as the stored big-endian word loads) for both image forms:
//   round 5: 15 table steps, the sets of build_fold_nibbles_pre (the fold carries the last step);
//   round 4: 16 table steps, the sets of build_fold_nibbles (lab variant 157).
// The reference CRC is the byte-at-a-time SWCrc32c loop (src/common/SWCrc32c.cpp:97-104).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "crc32c_tables.h"

using namespace hdfs3crc;

namespace {

uint32_t sw_crc(const uint32_t t0[256], const uint8_t *p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) c = t0[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    return ~c;
}

uint32_t step(const uint32_t t[kSlices][kTableEntries], uint32_t x) {  // Lut::word(x, 0)
    return t[3][x & 0xFFu] ^ t[2][(x >> 8) & 0xFFu] ^ t[1][(x >> 16) & 0xFFu] ^ t[0][x >> 24];
}

int check(const uint32_t t[kSlices][kTableEntries], const std::vector<uint32_t> &fold, bool pre, const uint8_t *round) {
    int bad = 0;
    for (int set = 0; set < 4; ++set) {
        const int g = kFoldGs[set];
        const uint32_t *nib = fold.data() + (pre ? kFoldAffineOff : kFoldAffineOldOff) + set * kFoldNibbleWords;
        for (int chunk = 0; chunk < 64 / g; ++chunk) {
            uint32_t y = 0;
            for (int j = 0; j < g; ++j) {
                const int lane = chunk * g + j;
                uint32_t w[16];
                std::memcpy(w, round + 64 * lane, 64);  // little-endian dwords, as the GPU loads them
                uint32_t x = w[0];
                for (int i = 1; i < 16; ++i) x = step(t, x) ^ w[i];
                if (!pre) x = step(t, x);  // round 4: the chain's last table step, then the fold
                for (int k = 0; k < 8; ++k) y ^= nib[(k * 16 + ((x >> (4 * k)) & 15u)) * 64 + lane];
            }
            const uint32_t want = __builtin_bswap32(sw_crc(t[0], round + 64 * g * chunk, size_t(64) * g));
            if (y != want) {
                if (bad < 5)
                    std::printf("MISMATCH pre=%d G=%d chunk=%d got %08x want %08x\n", int(pre), g, chunk, y, want);
                ++bad;
            }
        }
    }
    return bad;
}

}  // namespace

int main() {
    int bad = 0;
    const uint32_t polys[2] = {kPolyReflected, kPolyCrc32};
    for (uint32_t poly : polys) {
        static uint32_t t[kSlices][kTableEntries];
        build_slice_tables(t, poly);
        std::vector<uint32_t> fold(kFoldImageWords);
        build_fold_matrices(t[0], fold.data());
        for (int set = 0; set < 4; ++set) {  // as hdfs3_crc.cpp host_images builds them
            uint32_t *nib = fold.data() + kFoldAffineOff + set * kFoldNibbleWords;
            build_fold_nibbles_pre(t[0], fold.data(), set, nib);
            build_fold_affine(t[0], set, nib);
            uint32_t *old = fold.data() + kFoldAffineOldOff + set * kFoldNibbleWords;
            build_fold_nibbles(fold.data(), set, old);
            build_fold_affine(t[0], set, old);
        }
        std::mt19937_64 rng(poly);
        std::vector<uint8_t> round(4096);
        for (int r = 0; r < 24; ++r) {
            for (auto &b : round) b = uint8_t(rng());
            if (r == 0) std::memset(round.data(), 0, round.size());
            if (r == 1) std::memset(round.data(), 0xFF, round.size());
            bad += check(t, fold, true, round.data());
            bad += check(t, fold, false, round.data());
        }
    }
    if (bad) {
        std::printf("%d mismatching chunks\n", bad);
        return 1;
    }
    std::printf("fold image ok\n");
    return 0;
}
