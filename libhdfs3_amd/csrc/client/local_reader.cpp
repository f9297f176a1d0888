// hdfs3_local_reader: LocalBlockReader (src/client/LocalBlockReader.cpp) — the short-
// circuit read of a block file and its .meta file — with readAndVerify's per-chunk CPU
// loop (:138-163) replaced by GPU verification of large windows.
//
// .meta layout (:40-43, :64-121): BE16 version (1) | u8 checksum type | BE32 bytesPerChecksum
// | one BE32 CRC per chunk. Local semantics check every chunk, the short tail included.
//
// Pipeline: a loader thread preads a window (window_buffers x buffer_size bytes of block
// data, chunk aligned) and its CRC words into a pinned arena, then queues H2D + verify
// (check_short_tail=1) + result D2H + event on the ctx stream; the caller's read() waits
// for a window's event and copies verified bytes out, while the loader fills the next.
// Delivery granularity on a mismatch is the reference's: readAndVerify verifies one
// buffer_size buffer before any of it is returned, so bytes of the buffer holding the
// first bad chunk — and everything after — are withheld and -EIO is returned.
//
// Staging. Verification on: a window is pread into its pinned arena by the loader and the
// helper threads together (a single pread thread was the single-stream limit), DMA'd, and
// copied out. Verification off: the block file is mmap'd (MappedFileWrapper, MappedFileWrapper.cpp:
// 58-70, is the reference's own mmap reader) and read() copies straight out of the page cache,
// one copy per byte. HDFS3_LOCAL_MMAP=1 also maps verified reads: each window's page-cache pages
// are registered with HIP (pinned in place) and DMA'd directly, then copied out of the mapping;
// registration pins at ~23 GiB/s and serialises across threads in the runtime, so it is an
// opt-in (docs/DESIGN_HISTORY.md §5.1). HDFS3_LOCAL_MMAP=0 disables mapping altogether. Any mmap or
// registration failure falls back to the pread path for that window or reader.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../copy_pool.h"
#include "../ctx.h"
#include "../numa.h"
#include "hdfs3_client.h"
#include "hdfs3_crc.h"
#include "wire.h"

using namespace hdfs3crc;

namespace {

constexpr int kMetaHeader = 7;             // HEADER_SIZE: version 2 + type 1 + bpc 4
constexpr int kSlots = 3;
constexpr int32_t kDefaultBuffer = 1 << 20;  // input.localread.default.buffersize
constexpr int kDefaultWindowBuffers = 4;  // 4 MiB windows: first delivery sooner (docs/DESIGN_HISTORY.md §5.1)
constexpr int32_t kMaxBuffer = 1 << 30;     // largest local buffer / window

// Window events: HDFS3_LOCAL_BLOCKING_SYNC=1 makes the consumer sleep in hipEventSynchronize
// (hipEventBlockingSync) instead of spinning, leaving the cores to the copies when many readers
// run at once (round 4 measurement knob; the default keeps the spin)
unsigned window_event_flags() {
    static const unsigned f = [] {
        const char *e = getenv("HDFS3_LOCAL_BLOCKING_SYNC");
        return unsigned(hipEventDisableTiming) | (e && e[0] == '1' ? unsigned(hipEventBlockingSync) : 0u);
    }();
    return f;
}

int hip_err(hipError_t e, const char *what) {
    return fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

#define HIP_OK(expr)                                      \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_err(e_, #expr);  \
    } while (0)

// Reader resources — a ctx (stream, table images) and kSlots pinned + device windows —
// are pooled per process. The reference opens one LocalBlockReader per block
// (InputStreamImpl::setupBlockReader), and creating a ctx and pinning the windows costs
// more than reading a 128 MiB block from the page cache (docs/DESIGN_HISTORY.md §5.1).
struct LocalResources {
    hdfs3_crc_ctx *ctx = nullptr;
    PacketArena a[kSlots];
};
std::mutex g_pool_mu;
std::vector<LocalResources> g_pool;
constexpr size_t kPoolMax = 16;

bool take_pooled(int device, size_t cap, LocalResources *out) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_pool.size(); ++i) {
        if (g_pool[i].ctx->device == device && g_pool[i].a[0].cap >= cap) {
            *out = g_pool[i];
            g_pool.erase(g_pool.begin() + long(i));
            return true;
        }
    }
    return false;
}

void free_resources(LocalResources &r) {
    for (PacketArena &a : r.a) a.release();
    ctx_release(r.ctx);
    r.ctx = nullptr;
}

// pinned / device bytes of a pooled entry: its windows and what its ctx holds
LocalPoolStats entry_bytes(const LocalResources &r) {
    LocalPoolStats st;
    ctx_footprint(r.ctx, &st.pinned, &st.device);
    for (const PacketArena &a : r.a) {
        const uint64_t n = a.cap + (a.h_res ? sizeof(unsigned long long) : 0);
        st.pinned += n;
        st.device += n;
    }
    st.entries = 1;
    return st;
}

// a pooled entry dropped to keep the cap: destroyed outright, as local_pool_trim does. Releasing its
// ctx into the ctx pool would only move the bytes the cap just refused into the other pool.
void destroy_resources(LocalResources &r) {
    for (PacketArena &a : r.a) a.release();
    hdfs3_crc_ctx_destroy(r.ctx);
    r.ctx = nullptr;
}

// Pooled unless that would take the retained pinned bytes of both pools past the cap
// (HDFS3_POOL_PINNED_MAX): the oldest pooled entries are evicted first, then this one is not
// admitted. The decision is made under pool_admission_mu (ctx.h), so a ctx_release or another
// give_back on another thread cannot admit bytes into the same headroom meanwhile.
void give_back(LocalResources r) {
    std::vector<LocalResources> evict;
    bool keep = false;
    {
        std::lock_guard<std::mutex> adm(pool_admission_mu());
        const uint64_t cap = pool_pinned_cap_bytes(), ctxs = ctx_pool_pinned_bytes(), mine = entry_bytes(r).pinned;
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (g_pool.size() < kPoolMax) {
            uint64_t local = 0;
            for (const LocalResources &e : g_pool) local += entry_bytes(e).pinned;
            while (!g_pool.empty() && ctxs + local + mine > cap) {
                local -= entry_bytes(g_pool.front()).pinned;
                evict.push_back(g_pool.front());
                g_pool.erase(g_pool.begin());
            }
            if (ctxs + local + mine <= cap) {
                g_pool.push_back(r);
                keep = true;
            }
        }
    }
    for (LocalResources &e : evict) destroy_resources(e);
    // not admitted: the windows go, and the ctx takes its own admission into the ctx pool
    // (ctx_release takes pool_admission_mu itself, so this runs after the scope above)
    if (!keep) free_resources(r);
}

// Copies out of a verified window (one thread ~11 GiB/s) and the window preads (one thread
// ~9-12 GiB/s) are this reader's single-stream limits: both go through the process-wide
// CopyPool (copy_pool.h).

struct Window {
    PacketArena a;            // h/d: [data (cap_data)][crc words]
    int64_t start = 0;        // block offset of the window's first byte (chunk aligned)
    uint32_t len = 0;         // data bytes
    int64_t bad_chunk = -1;   // first mismatching chunk (block-relative), after wait
    bool verified = false;
    const uint8_t *src = nullptr;  // where read() copies from: a.h, or the mapping
    void *reg = nullptr;           // mapped mode: the window's registered page range
};

constexpr int64_t kPage = 4096;

}  // namespace

namespace hdfs3crc {
LocalPoolStats local_pool_stats() {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    LocalPoolStats st;
    for (const LocalResources &e : g_pool) {
        const LocalPoolStats b = entry_bytes(e);
        st.pinned += b.pinned;
        st.device += b.device;
        st.entries += 1;
    }
    return st;
}

int local_pool_trim() {
    std::vector<LocalResources> idle;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        idle.swap(g_pool);
    }
    // destroyed outright, not released: a trim leaves no context behind in either pool
    for (LocalResources &e : idle) {
        for (PacketArena &a : e.a) a.release();
        hdfs3_crc_ctx_destroy(e.ctx);
    }
    return int(idle.size());
}
}  // namespace hdfs3crc

struct hdfs3_local_reader {
    int data_fd = -1, meta_fd = -1;
    hdfs3_crc_ctx *ctx = nullptr;
    bool verify = true;
    int checksum_type = 2;
    uint32_t flags = 0;                      // hdfs3_local_opts.flags
    uint32_t chunk_size = 0;
    int32_t buffer_size = kDefaultBuffer;    // localBufferSize (chunk-rounded when verifying)
    uint32_t window = 0;                     // bytes per GPU window (multiple of buffer_size)
    size_t cap_data = 0;
    int64_t length = 0;                      // block length
    int64_t first = 0;                       // first byte the loader reads (chunk aligned)
    int64_t cursor = 0;                      // next byte handed to the caller

    std::mutex mu;
    std::condition_variable cv;
    Window slot[kSlots];
    std::deque<int> ready, free_slots;
    bool load_done = false, stop = false;
    int load_error = 0;
    std::string load_msg;
    std::thread loader;
    int error = 0;
    std::string error_msg;
    std::atomic<uint64_t> batches{0};
    // mapped mode
    uint8_t *map = nullptr;
    size_t map_len = 0;                      // length rounded up to a page
    bool map_verified = false;               // HDFS3_LOCAL_MMAP=1: verified windows DMA'd from the mapping
    std::atomic<uint64_t> mapped_windows{0};

    int sticky(int code, const std::string &msg) {
        error = code;
        error_msg = msg;
        return fail(code, "%s", msg.c_str());
    }

    // LocalBlockReader ctor (:46-130): meta header, engine selection, buffer size
    int open_meta(bool want_verify) {
        uint8_t h[kMetaHeader];
        if (int rc = pread_fully(meta_fd, h, sizeof(h), 0)) return sticky(rc, "LocalBlockReader: cannot read the meta header");
        const int version = (h[0] << 8) | h[1];
        if (version != 1)
            return sticky(-EIO, "LocalBlockReader get an unmatched block, expected block version 1, real version is " +
                                    std::to_string(version));
        checksum_type = h[2];
        verify = want_verify;
        switch (checksum_type) {
        case wire::kChecksumNull: verify = false; break;
        case wire::kChecksumCrc32c:
        case wire::kChecksumCrc32:
            // Both types select the CRC32C engine (:85-98), as in the reference: a block
            // whose meta declares CHECKSUM_CRC32 is verified with CRC32C and so fails with
            // ChecksumException there and here. HDFS3_LOCAL_CRC32_AS_ZLIB opts into the
            // polynomial the meta declares instead (see engine_type()).
            chunk_size = (uint32_t(h[3]) << 24) | (uint32_t(h[4]) << 16) | (uint32_t(h[5]) << 8) | h[6];
            break;
        default:
            return sticky(-EIO, "LocalBlockReader cannot recognize checksum type: " + std::to_string(checksum_type));
        }
        // LocalBlockReader.cpp:100-115 reads bytesPerChecksum as a signed int and rejects only
        // chunkSize <= 0; a chunk above 1 GiB then fails the local buffer bound at open
        if (verify && (chunk_size == 0 || chunk_size > uint32_t(INT32_MAX)))
            return sticky(-EIO, "LocalBlockReader get an invalid checksum parameter, bytes per check: " +
                                    std::to_string(chunk_size));
        return 0;
    }

    // the polynomial the GPU checks this block with
    int engine_type() const {
        return checksum_type == wire::kChecksumCrc32 && (flags & HDFS3_LOCAL_CRC32_AS_ZLIB) ? HDFS3_CHECKSUM_TYPE_CRC32
                                                                                          : HDFS3_CHECKSUM_TYPE_CRC32C;
    }

    // ---- loader thread ------------------------------------------------------------------
    int load(Window &w, int64_t start) {
        w.start = start;
        w.len = uint32_t(std::min<int64_t>(window, length - start));
        w.bad_chunk = -1;
        w.verified = false;
        w.src = w.a.h;
        w.reg = nullptr;
        const uint8_t *h2d_src = w.a.h;
        if (map && !verify) {
            w.src = map + start;  // no staging at all: read() copies from the page cache
        } else if (map && map_verified && start % kPage == 0) {
            // pin the window's page-cache pages in place; the DMA reads them directly
            const size_t reg_len = size_t(std::min<int64_t>((start + w.len + kPage - 1) / kPage * kPage,
                                                            int64_t(map_len)) - start);
            if (hipHostRegister(map + start, reg_len, hipHostRegisterReadOnly) == hipSuccess) {
                w.reg = map + start;
                w.src = h2d_src = map + start;
                mapped_windows.fetch_add(1, std::memory_order_relaxed);
            } else {
                (void)hipGetLastError();  // pread path for this window
            }
        }
        if (w.src == w.a.h) {
            if (int rc = CopyPool::get().pread(data_fd, w.a.h, w.len, start)) {
                load_msg = "LocalBlockReader: failed to read the block file";
                return rc;
            }
        }
        batches.fetch_add(1, std::memory_order_relaxed);
        if (!verify) {
            w.verified = true;
            return 0;
        }
        const uint64_t chunk0 = uint64_t(start) / chunk_size;
        const uint64_t chunks = (uint64_t(w.len) + chunk_size - 1) / chunk_size;
        if (int rc = pread_fully(meta_fd, w.a.h + cap_data, 4 * chunks, kMetaHeader + 4 * int64_t(chunk0))) {
            load_msg = "LocalBlockReader: failed to read the meta file";
            return rc;
        }
        HIP_OK(hipMemcpyAsync(w.a.d, h2d_src, w.len, hipMemcpyHostToDevice, ctx->stream));
        HIP_OK(hipMemcpyAsync(w.a.d + cap_data, w.a.h + cap_data, 4 * chunks, hipMemcpyHostToDevice, ctx->stream));
        HIP_OK(hipMemsetAsync(w.a.d_res, 0, sizeof(unsigned long long), ctx->stream));
        if (int rc = hdfs3_crc32c_verify_dev_async(ctx, w.a.d, w.len, chunk_size, w.a.d + cap_data,
                                                   /*check_short_tail=*/1, reinterpret_cast<uint64_t *>(w.a.d_res))) {
            load_msg = hdfs3_crc_last_error();
            return rc;
        }
        HIP_OK(hipMemcpyAsync(w.a.h_res, w.a.d_res, sizeof(unsigned long long), hipMemcpyDeviceToHost, ctx->stream));
        HIP_OK(hipEventRecord(w.a.done, ctx->stream));
        return 0;
    }

    void run_loader() {
        (void)hipSetDevice(ctx->device);
        bind_thread_to_device(ctx->device);  // preads land next to the GPU (numa.h)
        int64_t next = first;
        while (next < length) {
            int s;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !free_slots.empty(); });
                if (stop) return;
                s = free_slots.front();
                free_slots.pop_front();
            }
            const int rc = load(slot[s], next);
            {
                std::lock_guard<std::mutex> lk(mu);
                if (rc) {
                    load_error = rc;
                    if (load_msg.empty()) load_msg = hdfs3_crc_last_error();
                    free_slots.push_back(s);
                } else {
                    ready.push_back(s);
                }
                if (rc || next + slot[s].len >= length) load_done = true;
            }
            cv.notify_all();
            if (rc) return;
            next += slot[s].len;
        }
        std::lock_guard<std::mutex> lk(mu);
        load_done = true;
        cv.notify_all();
    }

    void release_pages(Window &w) {
        if (w.reg) {
            (void)hipHostUnregister(w.reg);
            w.reg = nullptr;
        }
    }

    // ---- caller side ----------------------------------------------------------------------
    int wait(Window &w) {
        if (w.verified) return 0;
        HIP_OK(hipEventSynchronize(w.a.done));
        const unsigned long long r = *w.a.h_res;
        if (r) w.bad_chunk = int64_t(uint64_t(w.start) / chunk_size) + hdfs3_crc_decode_result(r);
        w.verified = true;
        return 0;
    }

    int32_t read(uint8_t *out, int32_t len) {
        if (error) return fail(error, "%s", error_msg.c_str());
        if (!out || len <= 0) return fail(-EINVAL, "invalid read buffer");
        int32_t total = 0;
        while (total < len && cursor < length) {
            int s;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !ready.empty() || load_done; });
                if (ready.empty()) {
                    if (load_error) {
                        const int code = load_error;
                        const std::string msg = load_msg;
                        lk.unlock();
                        if (total) {
                            error = code;
                            error_msg = msg;
                            return total;
                        }
                        return sticky(code, msg);
                    }
                    break;
                }
                s = ready.front();
            }
            Window &w = slot[s];
            if (int rc = wait(w)) return total ? total : sticky(rc, hdfs3_crc_last_error());
            // deliverable end: everything, or up to the local buffer holding the bad chunk
            int64_t end = w.start + w.len;
            if (w.bad_chunk >= 0) {
                const int64_t bad_off = w.bad_chunk * int64_t(chunk_size);
                end = first + (bad_off - first) / buffer_size * int64_t(buffer_size);
            }
            const int64_t begin = std::max<int64_t>(cursor, w.start);
            if (begin < end) {
                const int64_t n = std::min<int64_t>(end - begin, len - total);
                CopyPool::get().copy(out + total, w.src + (begin - w.start), size_t(n));
                total += int32_t(n);
                cursor = begin + n;
            }
            if (w.bad_chunk >= 0 && cursor >= end) {
                sticky(-EIO, "ChecksumException: LocalBlockReader checksum not match for block (chunk " +
                                 std::to_string(w.bad_chunk) + ")");
                return total ? total : error;
            }
            if (cursor >= w.start + w.len) {
                release_pages(w);  // its DMA completed: wait() saw the event
                {
                    std::lock_guard<std::mutex> lk(mu);
                    ready.pop_front();
                    free_slots.push_back(s);
                }
                cv.notify_all();
            }
        }
        return total;
    }

    int64_t available() {
        std::lock_guard<std::mutex> lk(mu);
        int64_t a = 0;
        for (int s : ready)
            if (slot[s].verified && slot[s].bad_chunk < 0)
                a += slot[s].start + slot[s].len - std::max<int64_t>(cursor, slot[s].start);
        return a;
    }

    ~hdfs3_local_reader() {
        if (loader.joinable()) {
            {
                std::lock_guard<std::mutex> lk(mu);
                stop = true;
            }
            cv.notify_all();
            loader.join();
        }
        if (ctx) {
            LocalResources res;
            res.ctx = ctx;
            for (int i = 0; i < kSlots; ++i) res.a[i] = slot[i].a;
            // a ctx whose stream completes cleanly goes back to the pool for the next reader
            const bool clean = hipStreamSynchronize(ctx->stream) == hipSuccess;
            for (Window &w : slot) release_pages(w);  // no DMA is in flight any more
            if (clean && res.a[kSlots - 1].done)
                give_back(res);
            else
                free_resources(res);
        }
        if (map) munmap(map, map_len);
        if (data_fd >= 0) ::close(data_fd);
        if (meta_fd >= 0) ::close(meta_fd);
    }
};

extern "C" {

int hdfs3_local_reader_open(const char *data_path, const char *meta_path, int64_t num_bytes, int64_t offset,
                            const hdfs3_local_opts *opts, hdfs3_local_reader **out) {
    if (!out || !data_path || !meta_path || offset < 0) return fail(-EINVAL, "invalid argument");
    *out = nullptr;
    hdfs3_local_reader *r = new (std::nothrow) hdfs3_local_reader();
    if (!r) return fail(-ENOMEM, "reader allocation");
    auto bail = [&](int rc) {
        delete r;
        return rc;
    };
    const int device = opts ? opts->device : 0;
    if (opts && opts->buffer_size > 0) r->buffer_size = opts->buffer_size;
    if (opts) r->flags = opts->flags;
    if (opts && (opts->flags & ~HDFS3_LOCAL_CRC32_AS_ZLIB)) return bail(fail(-EINVAL, "unknown local reader flags"));
    const int wbuf = opts && opts->window_buffers > 0 ? opts->window_buffers : kDefaultWindowBuffers;
    r->data_fd = ::open(data_path, O_RDONLY | O_CLOEXEC);
    if (r->data_fd < 0) return bail(fail(-errno, "LocalBlockReader: cannot open block file %s", data_path));
    r->meta_fd = ::open(meta_path, O_RDONLY | O_CLOEXEC);
    if (r->meta_fd < 0) return bail(fail(-errno, "LocalBlockReader: cannot open meta file %s", meta_path));
    struct stat st;
    if (fstat(r->data_fd, &st) != 0) return bail(fail(-errno, "fstat failed"));
    r->length = num_bytes > 0 ? num_bytes : int64_t(st.st_size);
    if (num_bytes > int64_t(st.st_size)) return bail(fail(-EIO, "block file shorter than the block length"));
    if (offset > r->length) return bail(fail(-EINVAL, "offset beyond the block"));
    if (int rc = r->open_meta(opts ? opts->verify != 0 : true)) return bail(rc);
    if (r->verify) {  // chunk-rounded local buffer (:112-116); reads start on a chunk (skip, :232-263)
        const int64_t rounded = (int64_t(r->buffer_size) + r->chunk_size - 1) / r->chunk_size * r->chunk_size;
        if (rounded > kMaxBuffer)
            return bail(fail(-EINVAL, "LocalBlockReader: local buffer of %lld bytes (chunk-rounded) exceeds %d",
                             (long long)rounded, kMaxBuffer));
        r->buffer_size = int32_t(rounded);
        r->first = offset / r->chunk_size * r->chunk_size;
    } else {
        if (r->buffer_size > kMaxBuffer) return bail(fail(-EINVAL, "LocalBlockReader: local buffer above 1 GiB"));
        r->first = offset;
    }
    r->cursor = offset;
    // whole buffers per window, at least one (the buffer itself is at most 1 GiB)
    r->window = uint32_t(std::max<int64_t>(1, std::min<int64_t>(wbuf, kMaxBuffer / r->buffer_size)) * r->buffer_size);
    // mapped mode: verification off always (copies straight from the page cache); verified
    // reads only with HDFS3_LOCAL_MMAP=1, and only when every window starts on a page (first
    // and the window size page multiples), so windows register disjoint page ranges
    const char *mm = getenv("HDFS3_LOCAL_MMAP");
    r->map_verified = mm && mm[0] == '1' && r->verify && r->first % kPage == 0 && r->window % kPage == 0;
    if (r->length > 0 && !(mm && mm[0] == '0') && (!r->verify || r->map_verified)) {
        r->map_len = size_t((r->length + kPage - 1) / kPage * kPage);
        void *m = mmap(nullptr, r->map_len, PROT_READ, MAP_SHARED, r->data_fd, 0);
        if (m != MAP_FAILED) {
            r->map = static_cast<uint8_t *>(m);
            (void)madvise(m, r->map_len, MADV_SEQUENTIAL);
        } else {
            r->map_len = 0;
        }
    }
    r->cap_data = (size_t(r->window) + 255) & ~size_t(255);
    const size_t crc_bytes = r->verify ? 4 * ((size_t(r->window) + r->chunk_size - 1) / r->chunk_size) : 0;
    // the windows live on `device`, whatever the calling thread's current device is
    DeviceGuard guard(device);
    LocalResources pooled;
    if (take_pooled(device, r->cap_data + crc_bytes, &pooled)) {
        r->ctx = pooled.ctx;
        for (int i = 0; i < kSlots; ++i) r->slot[i].a = pooled.a[i];
    } else {
        if (int rc = ctx_acquire(device, &r->ctx)) return bail(rc);
        // the windows are pinned from a thread bound to the GPU's NUMA node (numa.h), so the
        // block file's pages are read into memory next to the GPU that DMAs them
        bool ok = true;
        auto alloc_windows = [&] {
            for (Window &w : r->slot) {
                PacketArena &a = w.a;
                if (hipHostMalloc(reinterpret_cast<void **>(&a.h), r->cap_data + crc_bytes, pinned_host_flags()) !=
                        hipSuccess ||
                    hipMalloc(reinterpret_cast<void **>(&a.d), r->cap_data + crc_bytes) != hipSuccess ||
                    hipMalloc(reinterpret_cast<void **>(&a.d_res), sizeof(unsigned long long)) != hipSuccess ||
                    hipHostMalloc(reinterpret_cast<void **>(&a.h_res), sizeof(unsigned long long),
                                  pinned_host_flags()) != hipSuccess ||
                    hipEventCreateWithFlags(&a.done, window_event_flags()) != hipSuccess) {
                    ok = false;
                    return;
                }
                a.cap = r->cap_data + crc_bytes;
            }
        };
        if (!numa_binding_enabled()) {
            alloc_windows();  // binding off (the default): the caller's thread, under the guard
        } else {
            try {
                std::thread([&] {
                    (void)hipSetDevice(device);
                    bind_thread_to_device(device);
                    alloc_windows();
                }).join();
            } catch (const std::system_error &) {
                ok = false;  // no thread: never let the exception cross the extern "C" entry point
            }
        }
        if (!ok) return bail(fail(-ENOMEM, "LocalBlockReader: window allocation failed"));
    }
    if (int rc = hdfs3_crc_ctx_set_checksum_type(r->ctx, r->engine_type())) return bail(rc);
    for (int i = 0; i < kSlots; ++i) r->free_slots.push_back(i);
    if (r->first < r->length) {
        r->loader = std::thread([r] { r->run_loader(); });
    } else {
        r->load_done = true;
    }
    *out = r;
    return 0;
}

int32_t hdfs3_local_reader_read(hdfs3_local_reader *r, void *buf, int32_t len) {
    if (!r) return fail(-EINVAL, "null reader");
    return r->read(static_cast<uint8_t *>(buf), len);
}

int64_t hdfs3_local_reader_available(hdfs3_local_reader *r) { return r ? r->available() : 0; }

int hdfs3_local_reader_stats(hdfs3_local_reader *r, uint32_t *bpc, int *checksum_type, uint64_t *gpu_batches) {
    if (!r) return fail(-EINVAL, "null reader");
    if (bpc) *bpc = r->chunk_size;
    if (checksum_type) *checksum_type = r->checksum_type;
    if (gpu_batches) *gpu_batches = r->batches.load();
    return 0;
}

uint64_t hdfs3_local_reader_mapped_windows(hdfs3_local_reader *r) { return r ? r->mapped_windows.load() : 0; }

int hdfs3_local_reader_close(hdfs3_local_reader *r) {
    delete r;
    return 0;
}

}  // extern "C"
