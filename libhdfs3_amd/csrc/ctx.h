// Internal: the hdfs3_crc_ctx definition, shared by the C-ABI (hdfs3_crc.cpp) and the
// block reader (client/block_reader.cpp). Not installed.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>

#include "crc32c_kernels.h"

namespace hdfs3crc {

// Sets the thread-local message returned by hdfs3_crc_last_error(); returns `code`.
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// Makes `dev` the calling thread's current device for the guard's lifetime (hipMalloc,
// hipHostMalloc and event creation act on the current device).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
        else prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// Staging segment of the host-buffer API: 16 MiB of payload per H2D transfer.
constexpr size_t kSegmentBytes = 16u << 20;

struct Slot {
    uint8_t *h_data = nullptr, *h_crc = nullptr;  // pinned
    uint8_t *d_data = nullptr, *d_crc = nullptr;  // device
    size_t data_cap = 0, crc_cap = 0;
    hipEvent_t done = nullptr;
    // compute: CRC bytes waiting in h_crc to be copied out once `done` fires
    uint8_t *pending_out = nullptr;
    size_t pending_bytes = 0;
};

// One packet batch's buffers for the block reader: pinned wire arena + its HBM mirror,
// packet descriptors, the verify result word and the completion event. Cached in the ctx
// so the block readers an input stream opens one after another reuse them.
struct PacketArena {
    uint8_t *h = nullptr, *d = nullptr;
    size_t cap = 0;
    DevSegment *h_desc = nullptr, *d_desc = nullptr;  // descriptor staging (DevSegment-sized)
    size_t desc_cap = 0;
    unsigned long long *d_res = nullptr, *h_res = nullptr;
    hipEvent_t done = nullptr;
    // 4096-byte piece CRCs of a batch at bpc = R x 4096 (launch_chunks' pieces + combine): the
    // batch's own, so two readers verifying on one ctx (a stream's sequential reader and a pread's)
    // never share it (round 5; the ctx's scratch is for the calls of the ctx's own thread)
    PieceScratch pieces;

    void release() {
        pieces.release();
        if (h) (void)hipHostFree(h);
        if (d) (void)hipFree(d);
        if (h_desc) (void)hipHostFree(h_desc);
        if (d_desc) (void)hipFree(d_desc);
        if (h_res) (void)hipHostFree(h_res);
        if (d_res) (void)hipFree(d_res);
        if (done) (void)hipEventDestroy(done);
        *this = PacketArena();
    }
};

}  // namespace hdfs3crc

struct hdfs3_crc_ctx;
namespace hdfs3crc {
// Process-wide pool of contexts for the client drop-ins (input/output streams, block and
// local readers). libhdfs3 opens a stream per file and a reader per block; creating a ctx
// (stream, table uploads, device query) and its pinned arenas costs milliseconds, more than
// reading a small file. A released ctx keeps its arena cache and goes back to the pool.
// acquire: a pooled ctx of `device` (stream reset to its own, type CRC32C) or a new one.
// deep = true: prefer the pooled ctx holding the most cached arenas (block read-ahead rings).
int ctx_acquire(int device, hdfs3_crc_ctx **out, bool deep = false);
// release: synchronizes the ctx's stream; pooled when that succeeds and the pool has room.
void ctx_release(hdfs3_crc_ctx *ctx);
// the pinned bytes the pool may retain (HDFS3_POOL_PINNED_MAX, default 1 GiB)
uint64_t pool_pinned_cap_bytes();
// pinned / device bytes a ctx holds beyond its tables (staging, cached arenas), and the pinned
// bytes the ctx pool retains now
void ctx_footprint(hdfs3_crc_ctx *ctx, uint64_t *pinned, uint64_t *device);
uint64_t ctx_pool_pinned_bytes();
// Serialises every ADMISSION into either pool (ctx_release, the local readers' give_back): the only
// operations that add retained pinned bytes. Each admission reads the other pool's bytes and decides
// under this lock, so two releases at once cannot both fit the same headroom. Taking a
// ctx or an entry out of a pool, shedding and trimming only lower the total and do not take it.
// Order: this lock first, then a pool's own mutex (never the reverse).
std::mutex &pool_admission_mu();
// The short-circuit readers' own pool (local_reader.cpp: a ctx and its windows per entry) counts
// against the same cap: its retained bytes, pooled entries, and a trim that frees them all
struct LocalPoolStats {
    uint64_t pinned = 0, device = 0, entries = 0;
};
LocalPoolStats local_pool_stats();
int local_pool_trim();
}  // namespace hdfs3crc

struct hdfs3_crc_ctx {
    int device = 0;
    int grid_cap = 256;            // one 1024-thread workgroup per CU (128 KiB LDS image)
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    uint32_t *d_tables = nullptr;  // active 4 x 256 slice-table image (checksum_type)
    uint32_t *d_fold = nullptr;    // active lane-fold GF(2) matrices (crc32c_tables.h)
    // per polynomial: [0] CRC32C (CHECKSUM_CRC32C = 2), [1] CRC-32/zlib (CHECKSUM_CRC32 = 1)
    uint32_t *d_tables_by[2] = {nullptr, nullptr};
    uint32_t *d_fold_by[2] = {nullptr, nullptr};
    int checksum_type = 2;
    uint32_t poly = 0x82F63B78u;        // reflected polynomial of checksum_type
    unsigned long long *d_result = nullptr;
    unsigned long long *h_result = nullptr;  // pinned
    // blocks API: a ring of descriptor stagings, each reusable once its event fired
    struct SegStage {
        hdfs3crc::DevSegment *h = nullptr, *d = nullptr;
        size_t cap = 0;
        hipEvent_t done = nullptr;
        bool armed = false;  // done recorded after a copy out of h that may still be pending
        hipEvent_t copied = nullptr;  // the descriptors' copy on desc_stream (DescCopy)
    } seg_ring[4];
    // long descriptor lists copy on this stream, beside the previous launch (DescCopy; created on first use)
    hipStream_t desc_stream = nullptr;
    unsigned seg_next = 0;
    hdfs3crc::WordScratch words;  // dense CRC words of compute over in-packet word regions
    hdfs3crc::PieceScratch pieces;  // 4096-byte piece CRCs of chunks above 4 KiB (launch_chunks)
    hdfs3crc::Slot slot[2];
    std::atomic<uint64_t> launches{0};
    std::mutex arena_mu;                          // guards arena_cache
    std::vector<hdfs3crc::PacketArena> arena_cache;
};

