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

constexpr uint32_t kPolyReflected = 0x82F63B78u;
constexpr int kSlices = 4;
constexpr int kTableEntries = 256;
constexpr int kTableWords = kSlices * kTableEntries;  // 1024 words = 4 KiB image

inline void build_slice_tables(uint32_t out[kSlices][kTableEntries]) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? kPolyReflected : 0u);
        out[0][i] = c;
    }
    for (int k = 1; k < kSlices; ++k)
        for (int i = 0; i < 256; ++i)
            out[k][i] = out[0][out[k - 1][i] & 0xFFu] ^ (out[k - 1][i] >> 8);
}

}  // namespace hdfs3crc
