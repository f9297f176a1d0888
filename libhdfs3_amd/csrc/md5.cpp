// MD5 per RFC 1321 §3.1-3.5: 64-byte blocks, four rounds of 16 steps over a
// little-endian message schedule, length padding in bits.
#include "md5.h"

#include <cstring>

namespace hdfs3crc {

namespace {

// K[i] = floor(2^32 * |sin(i + 1)|)
constexpr uint32_t kK[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

// per-round rotation amounts, 4 per round
constexpr int kS[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};

inline uint32_t rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

template <int I>
inline void step(uint32_t &a, uint32_t b, uint32_t c, uint32_t d, const uint32_t *m) {
    constexpr int round = I >> 4;
    constexpr int g = round == 0 ? I : round == 1 ? (5 * I + 1) & 15 : round == 2 ? (3 * I + 5) & 15 : (7 * I) & 15;
    // b is the previous step's result: everything that does not depend on it is summed first
    const uint32_t early = a + kK[I] + m[g];
    uint32_t t;
    if constexpr (round == 0) t = early + (d ^ (b & (c ^ d)));      // F = (b & c) | (~b & d)
    else if constexpr (round == 1) t = early + (c & ~d) + (b & d);  // G = (b & d) | (c & ~d), disjoint terms
    else if constexpr (round == 2) t = early + (b ^ (c ^ d));       // H
    else t = early + (c ^ (b | ~d));                                // I
    a = b + rotl(t, kS[round * 4 + (I & 3)]);
}

// four steps rotate the roles (a, b, c, d) -> (d, a, b, c); sixteen groups of four
template <int I>
inline void quad(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, const uint32_t *m) {
    step<I>(a, b, c, d, m);
    step<I + 1>(d, a, b, c, m);
    step<I + 2>(c, d, a, b, m);
    step<I + 3>(b, c, d, a, m);
    if constexpr (I + 4 < 64) quad<I + 4>(a, b, c, d, m);
}

void compress(uint32_t h[4], const uint8_t *blk) {
    uint32_t m[16];
    std::memcpy(m, blk, 64);  // little-endian words (x86 and the GPU box host are little-endian)
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    quad<0>(a, b, c, d, m);
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

}  // namespace

Md5::Md5() : h{0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476} {}

void Md5::update(const void *p, size_t n) {
    const uint8_t *s = static_cast<const uint8_t *>(p);
    total += n;
    if (fill) {
        const size_t take = n < 64 - fill ? n : 64 - fill;
        std::memcpy(buf + fill, s, take);
        fill += take;
        s += take;
        n -= take;
        if (fill < 64) return;
        compress(h, buf);
        fill = 0;
    }
    for (; n >= 64; s += 64, n -= 64) compress(h, s);
    if (n) {
        std::memcpy(buf, s, n);
        fill = n;
    }
}

void Md5::finish(uint8_t out[16]) {
    const uint64_t bits = total * 8;
    const uint8_t pad0 = 0x80;
    const uint8_t zeros[64] = {};
    update(&pad0, 1);
    update(zeros, fill <= 56 ? 56 - fill : 120 - fill);
    uint8_t len[8];
    for (int i = 0; i < 8; ++i) len[i] = uint8_t(bits >> (8 * i));
    update(len, 8);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = uint8_t(h[i] >> (8 * j));
}

}  // namespace hdfs3crc
