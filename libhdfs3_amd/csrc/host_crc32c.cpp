// Host CRC32C for the streaming `Checksum` shim (hdfs3_crc32c_update_host).
//
// Only sub-chunk pieces go through here: the partial chunk a writer carries
// across append() calls (src/client/OutputStreamImpl.cpp:309-314) and the
// Checksum ABC itself (src/common/Checksum.h:43-67). Every batch entry point of
// hdfs3_crc.h runs on the GPU and never calls this.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "crc32c_tables.h"

namespace hdfs3crc {
namespace {

struct HostTables {
    uint32_t t[4][256];
    HostTables() { build_slice_tables(t); }
};
const HostTables &tables() {
    static const HostTables h;
    return h;
}

__attribute__((target("sse4.2"))) uint32_t update_sse42(uint32_t c, const uint8_t *p, size_t n) {
    while (n && (reinterpret_cast<uintptr_t>(p) & 7u)) {
        c = __builtin_ia32_crc32qi(c, *p++);
        --n;
    }
    uint64_t c64 = c;
    for (; n >= 8; n -= 8, p += 8) {
        uint64_t v;
        std::memcpy(&v, p, 8);
        c64 = __builtin_ia32_crc32di(c64, v);
    }
    c = static_cast<uint32_t>(c64);
    while (n--) c = __builtin_ia32_crc32qi(c, *p++);
    return c;
}

uint32_t update_slice4(uint32_t c, const uint8_t *p, size_t n) {
    const auto &T = tables().t;
    for (; n >= 4; n -= 4, p += 4) {
        uint32_t w;
        std::memcpy(&w, p, 4);
        c ^= w;
        c = T[3][c & 0xFF] ^ T[2][(c >> 8) & 0xFF] ^ T[1][(c >> 16) & 0xFF] ^ T[0][c >> 24];
    }
    while (n--) c = T[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    return c;
}

}  // namespace

uint32_t host_update(uint32_t state, const void *p, size_t n) {
    static const bool have_sse42 = __builtin_cpu_supports("sse4.2");
    const uint8_t *b = static_cast<const uint8_t *>(p);
    return have_sse42 ? update_sse42(state, b, n) : update_slice4(state, b, n);
}

}  // namespace hdfs3crc
