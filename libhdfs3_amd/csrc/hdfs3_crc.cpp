// C-ABI of the MI355X CRC32C engine (include/hdfs3_crc.h).
//
// Error convention mirrors libhdfs3's C API (src/client/Hdfs.cpp:75-80,243-327):
// no exception crosses extern "C"; failures return a negative errno code and
// leave a thread-local message (hdfs3_crc_last_error, cf. hdfsGetLastError at
// Hdfs.cpp:59,329).
#include "hdfs3_crc.h"
#include "md5.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstddef>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <mutex>
#include <new>

#include "copy_pool.h"
#include "crc32c_kernels.h"
#include "crc32c_tables.h"
#include "ctx.h"
#include "numa.h"

namespace hdfs3crc {
uint32_t host_update(uint32_t state, const void *p, size_t n);
}

using namespace hdfs3crc;

namespace hdfs3crc {

thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

}  // namespace hdfs3crc

namespace hdfs3crc {

// Per polynomial ([0] CRC32C, [1] CRC32): slice tables, then the fold image (kFoldWords
// matrix columns, then the 4 affine nibble-table sets for G = 8, 16, 32, 64 of the round
// kernel), built once per process.
// the device copy: the product stops before the lab-only sets
#if HDFS3_LAB
constexpr size_t kFoldUploadBytes = sizeof(uint32_t) * kFoldImageWords;
#else
constexpr size_t kFoldUploadBytes = sizeof(uint32_t) * kFoldAffineOldOff;
#endif

struct HostImage {
    uint32_t t[kSlices][kTableEntries];
    uint32_t fold[kFoldImageWords];
};

const HostImage *host_images() {
    static HostImage img[2];
    static std::once_flag once;
    std::call_once(once, [] {
        const uint32_t polys[2] = {kPolyReflected, kPolyCrc32};
        for (int p = 0; p < 2; ++p) {
            build_slice_tables(img[p].t, polys[p]);
            build_fold_matrices(img[p].t[0], img[p].fold);
            for (int set = 0; set < 4; ++set) {
                uint32_t *nib = img[p].fold + kFoldAffineOff + set * kFoldNibbleWords;
                build_fold_nibbles_pre(img[p].t[0], img[p].fold, set, nib);
                build_fold_affine(img[p].t[0], set, nib);
#if HDFS3_LAB  // the round-4 sets of lab variant 157; the product never reads them (nor uploads them)
                uint32_t *old = img[p].fold + kFoldAffineOldOff + set * kFoldNibbleWords;
                build_fold_nibbles(img[p].fold, set, old);
                build_fold_affine(img[p].t[0], set, old);
#endif
            }
        }
    });
    return img;
}

}  // namespace hdfs3crc

namespace {

int hip_fail(hipError_t e, const char *what) {
    const int code = e == hipErrorOutOfMemory ? -ENOMEM
                     : e == hipErrorInvalidValue ? -EINVAL
                     : e == hipErrorNoDevice || e == hipErrorInvalidDevice ? -ENODEV
                                                                           : -EIO;
    return fail(code, "%s: %s", what, hipGetErrorString(e));
}

#define HIP_TRY(expr)                                  \
    do {                                               \
        hipError_t e_ = (expr);                        \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

}  // namespace

namespace {

int check_args(hdfs3_crc_ctx *ctx, uint32_t bpc) {
    if (!ctx) return fail(-EINVAL, "null hdfs3_crc_ctx");
    // any bytesPerChecksum > 0, as RemoteBlockReader::checkResponse accepts from a datanode
    // (RemoteBlockReader.cpp:150-156): sizes the whole-round kernels do not take (not 512..4096
    // or unaligned buffers) run on the byte-granular chunk-per-lane kernel
    if (bpc == 0) return fail(-EINVAL, "bytes per checksum must be positive");
    return 0;
}

int grow_slot(Slot &s, size_t data_bytes, size_t crc_bytes) {
    if (data_bytes > s.data_cap) {
        if (s.h_data) (void)hipHostFree(s.h_data);
        if (s.d_data) (void)hipFree(s.d_data);
        s.h_data = s.d_data = nullptr;
        s.data_cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.h_data), data_bytes, pinned_host_flags()));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&s.d_data), data_bytes));
        s.data_cap = data_bytes;
    }
    if (crc_bytes > s.crc_cap) {
        if (s.h_crc) (void)hipHostFree(s.h_crc);
        if (s.d_crc) (void)hipFree(s.d_crc);
        s.h_crc = s.d_crc = nullptr;
        s.crc_cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.h_crc), crc_bytes, pinned_host_flags()));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&s.d_crc), crc_bytes));
        s.crc_cap = crc_bytes;
    }
    return 0;
}

int finish_pending(Slot &s) {
    if (s.pending_out) {
        HIP_TRY(hipEventSynchronize(s.done));
        std::memcpy(s.pending_out, s.h_crc, s.pending_bytes);
        s.pending_out = nullptr;
        s.pending_bytes = 0;
    }
    return 0;
}

int launch(hdfs3_crc_ctx *ctx, const ChunkLaunch &in, bool verify) {
    ChunkLaunch a = in;
    HIP_TRY(launch_chunks(a, verify, ctx->d_tables, ctx->d_fold, ctx->grid_cap, ctx->stream, &ctx->pieces));
    ++ctx->launches;
    return 0;
}

// true when [p, p+len) is page-locked host memory the DMA engine can read directly
// (hdfs3_host_malloc_pinned, hipHostRegister); pageable memory is staged instead
bool is_pinned_host(const void *p) {
    hipPointerAttribute_t attr{};
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable pointers report an error; clear it
        return false;
    }
    return attr.type == hipMemoryTypeHost && attr.hostPointer != nullptr;
}

// Host-buffer pipeline shared by compute and verify: segments of whole chunks
// alternate between two pinned/device slots, so the CPU copy into pinned memory
// of segment i+1 overlaps the DMA and kernel of segment i.
int host_pipeline_impl(hdfs3_crc_ctx *ctx, const void *data, size_t len, uint32_t bpc,
                       const void *crc_in, void *crc_out, int check_short_tail,
                       int64_t *first_bad) {
    const bool verify = crc_in != nullptr;
    const size_t seg = (kSegmentBytes / bpc > 0 ? kSegmentBytes / bpc : 1) * size_t(bpc);
    const size_t seg_crc = (seg / bpc) * 4;
    if (verify) {
        HIP_TRY(hipMemsetAsync(ctx->d_result, 0, sizeof(unsigned long long), ctx->stream));
    }
    const uint8_t *src = static_cast<const uint8_t *>(data);
    const bool direct = is_pinned_host(data);  // skip the staging copy for pinned callers
    size_t off = 0;
    for (int k = 0; off < len; ++k) {
        Slot &s = ctx->slot[k & 1];
        const size_t n = len - off < seg ? len - off : seg;
        const size_t nc = (n + bpc - 1) / bpc;
        const size_t chunk0 = off / bpc;
        if (s.done) HIP_TRY(hipEventSynchronize(s.done));
        if (int rc = finish_pending(s)) return rc;
        if (int rc = grow_slot(s, seg, seg_crc)) return rc;
        if (!direct) CopyPool::get().copy(s.h_data, src + off, n);  // pageable: staged, split over the pool
        HIP_TRY(hipMemcpyAsync(s.d_data, direct ? src + off : s.h_data, n, hipMemcpyHostToDevice, ctx->stream));
        ChunkLaunch a{};
        a.data = s.d_data;
        a.len = n;
        a.bpc = bpc;
        a.chunk_base = chunk0;
        a.check_short_tail = check_short_tail;
        if (verify) {
            std::memcpy(s.h_crc, static_cast<const uint8_t *>(crc_in) + 4 * chunk0, 4 * nc);
            HIP_TRY(hipMemcpyAsync(s.d_crc, s.h_crc, 4 * nc, hipMemcpyHostToDevice, ctx->stream));
            a.crc_be = s.d_crc;
            a.result = ctx->d_result;
        } else {
            a.out_be = s.d_crc;
        }
        if (int rc = launch(ctx, a, verify)) return rc;
        if (!verify) {
            HIP_TRY(hipMemcpyAsync(s.h_crc, s.d_crc, 4 * nc, hipMemcpyDeviceToHost, ctx->stream));
            s.pending_out = static_cast<uint8_t *>(crc_out) + 4 * chunk0;
            s.pending_bytes = 4 * nc;
        }
        if (!s.done) HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(s.done, ctx->stream));
        off += n;
    }
    if (verify) {
        HIP_TRY(hipMemcpyAsync(ctx->h_result, ctx->d_result, sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (Slot &s : ctx->slot)
        if (int rc = finish_pending(s)) return rc;
    if (verify && first_bad) *first_bad = hdfs3_crc_decode_result(*ctx->h_result);
    return 0;
}

int host_pipeline(hdfs3_crc_ctx *ctx, const void *data, size_t len, uint32_t bpc,
                  const void *crc_in, void *crc_out, int check_short_tail,
                  int64_t *first_bad) {
    const int rc = host_pipeline_impl(ctx, data, len, bpc, crc_in, crc_out, check_short_tail, first_bad);
    if (rc != 0) {
        // a failed call must not leave CRC words queued for a caller buffer it no longer
        // owns: the next call would copy them out in finish_pending
        (void)hipStreamSynchronize(ctx->stream);
        for (Slot &sl : ctx->slot) sl.pending_out = nullptr;
    }
    return rc;
}

static_assert(sizeof(hdfs3_pkt_desc) == sizeof(DevPacket) && offsetof(hdfs3_pkt_desc, data_off) == offsetof(DevPacket, data_off) &&
                  offsetof(hdfs3_pkt_desc, crc_off) == offsetof(DevPacket, crc_off) &&
                  offsetof(hdfs3_pkt_desc, data_len) == offsetof(DevPacket, data_len),
              "the packets API hands descriptors to the kernels unconverted");

int stage_segments(hdfs3_crc_ctx *ctx, size_t n, hdfs3_crc_ctx::SegStage **out);

// One launch over n packets, nothing waited for: a single host pass over pk[] (bounds, layout
// detection, descriptors into a staging slot of the ctx's ring, which is reused only after its
// launch ran). Constant-pitch streams of whole-round packets take the wave kernel's pitch mode
// with no descriptor copy at all.
int packets_async(hdfs3_crc_ctx *ctx, const uint8_t *d_arena, size_t arena_len, const hdfs3_pkt_desc *pk, size_t n,
                  uint32_t bpc, bool verify, int check_short_tail, unsigned long long *d_result, bool overlap) {
    // the result key is (packet << 32 | chunk)
    if (n >= (size_t(1) << 31)) return fail(-EINVAL, "too many packets in one batch");
    hdfs3_crc_ctx::SegStage *st = nullptr;
    if (int rc = stage_segments(ctx, n, &st)) return rc;
    // hdfs3_pkt_desc and DevPacket share one layout (asserted above): no conversion copy
    const DevPacket *hp = reinterpret_cast<const DevPacket *>(pk);
    size_t bad = 0;
    bool staged = false;
    // a long list's descriptors copy on the ctx's side stream, under the launch before (the slot's
    // host and device halves are free: stage_segments waited for its last launch)
    DescCopy dc;
    if (n * sizeof(DevSegment) >= kSideCopyMinBytes) {
        if (!ctx->desc_stream) HIP_TRY(hipStreamCreateWithFlags(&ctx->desc_stream, hipStreamNonBlocking));
        if (!st->copied) HIP_TRY(hipEventCreateWithFlags(&st->copied, hipEventDisableTiming));
        dc.side = ctx->desc_stream;
        dc.copied = st->copied;
    }
    const hipError_t e = launch_packet_batch(d_arena, hp, n, bpc, verify, check_short_tail, d_result, st->h, st->d,
                                             ctx->d_tables, ctx->d_fold, ctx->grid_cap, ctx->stream, arena_len,
                                             &bad, overlap, &ctx->words, &ctx->pieces, &staged, &dc);
    if (e == hipErrorInvalidValue) return fail(-EINVAL, "packet %zu lies outside the %zu-byte arena", bad, arena_len);
    HIP_TRY(e);
    ++ctx->launches;
    // the launch copied its descriptors out of st->h asynchronously (the segmented kernel's array, the
    // chunk-per-lane kernel's DevPackets): the slot is reused only after that copy ran (round 5:
    // unarmed, a fifth async batch could overwrite a queued copy's source). A launch whose arguments
    // carried everything (the pitch walk: the writer's and the wire-layout batches) records nothing:
    // an event between barriered launches costs a marker packet, ~3 us of idle GPU (round 6)
    if (staged) {
        HIP_TRY(hipEventRecord(st->done, ctx->stream));
        st->armed = true;
    }
    return 0;
}

int packets_common(hdfs3_crc_ctx *ctx, const uint8_t *d_arena, size_t arena_len,
                   const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc, bool verify,
                   int check_short_tail, int64_t *bad_packet, int64_t *bad_chunk) {
    if (verify) HIP_TRY(hipMemsetAsync(ctx->d_result, 0, sizeof(unsigned long long), ctx->stream));
    if (int rc = packets_async(ctx, d_arena, arena_len, pk, n, bpc, verify, check_short_tail, ctx->d_result, false))
        return rc;
    if (verify) {
        HIP_TRY(hipMemcpyAsync(ctx->h_result, ctx->d_result, sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (verify) {
        const unsigned long long r = *ctx->h_result;
        const uint64_t key = r ? ~r : 0;
        if (bad_packet) *bad_packet = r ? int64_t(key >> 32) : -1;
        if (bad_chunk) *bad_chunk = r ? int64_t(key & 0xFFFFFFFFu) : -1;
    }
    return 0;
}

// hdfs3_pkt_stream: O(1) host work when the wave kernel's pitch mode takes the stream, else
// the descriptors are generated (once) and go through packets_async
int packet_stream_async(hdfs3_crc_ctx *ctx, const uint8_t *d_arena, size_t arena_len, const hdfs3_pkt_stream *ps,
                        uint32_t bpc, bool verify, int check_short_tail, unsigned long long *d_result, bool overlap) {
    if (ps->n == 0) return 0;
    if (ps->n >= (uint64_t(1) << 31)) return fail(-EINVAL, "too many packets in one stream");
    if (ps->last_len > ps->data_len) return fail(-EINVAL, "last_len above data_len");
    // bounds: the first and the last packet delimit the stream (pitch >= 0, offsets grow)
    const uint64_t last = ps->n - 1;
    const uint64_t lchunks = (uint64_t(ps->last_len) + bpc - 1) / bpc, chunks = (uint64_t(ps->data_len) + bpc - 1) / bpc;
    const unsigned __int128 ld = (unsigned __int128)ps->data_off + (unsigned __int128)last * ps->pitch;
    const unsigned __int128 lc = (unsigned __int128)ps->crc_off + (unsigned __int128)last * ps->pitch;
    if (ps->data_off + uint64_t(ps->n > 1 ? ps->data_len : ps->last_len) > arena_len || ld + ps->last_len > arena_len ||
        ps->crc_off + 4 * (ps->n > 1 ? chunks : lchunks) > arena_len || lc + 4 * lchunks > arena_len ||
        (ps->n > 1 && ps->pitch == 0))
        return fail(-EINVAL, "the packet stream does not fit the %zu-byte arena", arena_len);
    PacketGeom geom;
    if (packet_stream_ok(ps->data_len, ps->last_len, ps->n, bpc, d_arena + ps->data_off, d_arena + ps->crc_off,
                         ps->pitch, &geom)) {
        ChunkLaunch a{};
        a.data = d_arena + ps->data_off;
        a.crc_be = d_arena + ps->crc_off;
        a.out_be = const_cast<uint8_t *>(d_arena) + ps->crc_off;
        a.bpc = bpc;
        a.result = d_result;
        a.check_short_tail = check_short_tail;
        a.pitch = ps->pitch;
        a.npk = ps->n;
        a.geom = geom;
        a.last_len = ps->last_len;
        a.overlap_previous = overlap && verify;
        const hipError_t e =
            launch_packet_stream(a, verify, ctx->d_tables, ctx->d_fold, ctx->grid_cap, ctx->stream, &ctx->words,
                                 &ctx->pieces);
        if (e != hipErrorNotSupported) {
            HIP_TRY(e);
            ++ctx->launches;
            return 0;
        }
    }
    std::vector<hdfs3_pkt_desc> pk(ps->n);
    for (uint64_t i = 0; i < ps->n; ++i)
        pk[i] = hdfs3_pkt_desc{ps->data_off + i * ps->pitch, ps->crc_off + i * ps->pitch,
                               i == last ? ps->last_len : ps->data_len, 0};
    return packets_async(ctx, d_arena, arena_len, pk.data(), pk.size(), bpc, verify, check_short_tail, d_result, false);
}

// a descriptor staging slot of the blocks API, reusable once its previous launch ran
int stage_segments(hdfs3_crc_ctx *ctx, size_t n, hdfs3_crc_ctx::SegStage **out) {
    hdfs3_crc_ctx::SegStage &st = ctx->seg_ring[ctx->seg_next++ & 3u];
    if (st.armed) HIP_TRY(hipEventSynchronize(st.done));
    st.armed = false;
    if (n > st.cap) {
        if (st.h) (void)hipHostFree(st.h);
        if (st.d) (void)hipFree(st.d);
        st.h = st.d = nullptr;
        st.cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&st.h), n * sizeof(DevSegment), hipHostMallocDefault));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&st.d), n * sizeof(DevSegment)));
        st.cap = n;
    }
    if (!st.done) HIP_TRY(hipEventCreateWithFlags(&st.done, hipEventDisableTiming));
    *out = &st;
    return 0;
}

int blocks_common(hdfs3_crc_ctx *ctx, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc, bool verify,
                  int check_short_tail, unsigned long long *d_result) {
    if (n > (size_t(1) << 31)) return fail(-EINVAL, "too many blocks in one batch");
    for (size_t i = 0; i < n; ++i) {
        if (blocks[i].len && (!blocks[i].data || !blocks[i].crc_be)) return fail(-EINVAL, "block %zu: null buffer", i);
        if ((blocks[i].len + bpc - 1) / bpc >= (uint64_t(1) << 32))
            return fail(-EINVAL, "block %zu: 2^32 chunks or more", i);
    }
    hdfs3_crc_ctx::SegStage *st = nullptr;
    if (int rc = stage_segments(ctx, n, &st)) return rc;
    for (size_t i = 0; i < n; ++i)
        st->h[i] = DevSegment{static_cast<const uint8_t *>(blocks[i].data), static_cast<uint8_t *>(blocks[i].crc_be),
                              blocks[i].len, 0, uint64_t(i) << 32};
    // blocks of one 2-D tensor (constant data and word strides, equal whole-round blocks): the
    // wave kernel walks them directly (pitch mode); everything else: the segmented kernel
    const hipError_t te = launch_strided_blocks(st->h, n, bpc, verify, check_short_tail, d_result, ctx->d_tables,
                                                ctx->d_fold, ctx->grid_cap, ctx->stream, &ctx->words);
    if (te != hipErrorNotSupported) {
        HIP_TRY(te);
        ++ctx->launches;
    } else if (segments_fast(st->h, n, bpc)) {
        uint64_t uniform = 0;
        const uint64_t units = plan_segments(st->h, n, bpc, &uniform);
        if (n <= kMaxInlineSegments) {  // descriptors in the kernel arguments: no copy first
            HIP_TRY(launch_segments(nullptr, uint32_t(n), units, uniform, bpc, verify, check_short_tail, d_result,
                                    ctx->d_tables, ctx->d_fold, ctx->grid_cap, ctx->stream, st->h));
        } else {
            HIP_TRY(hipMemcpyAsync(st->d, st->h, n * sizeof(DevSegment), hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(launch_segments(st->d, uint32_t(n), units, uniform, bpc, verify, check_short_tail, d_result,
                                    ctx->d_tables, ctx->d_fold, ctx->grid_cap, ctx->stream));
            // the pinned staging is read by the copy: reusable once it ran. The other paths read
            // it on the host only (the launch's arguments carry what the kernel needs), and an
            // event between launches costs a marker packet (~4 us of idle between barriered
            // launches in the kernel trace of the batch pass, profiles/r03/prof/)
            HIP_TRY(hipEventRecord(st->done, ctx->stream));
            st->armed = true;
        }
        ++ctx->launches;
    } else {  // other chunk sizes or unaligned buffers: one launch per block, same keys
        for (size_t i = 0; i < n; ++i) {
            if (!blocks[i].len) continue;
            ChunkLaunch a{};
            a.data = st->h[i].data;
            a.len = blocks[i].len;
            a.bpc = bpc;
            a.crc_be = st->h[i].crc;
            a.out_be = st->h[i].crc;
            a.result = d_result;
            a.chunk_base = uint64_t(i) << 32;
            a.check_short_tail = check_short_tail;
            if (int rc = launch(ctx, a, verify)) return rc;
        }
    }
    return 0;
}

}  // namespace

extern "C" {

int hdfs3_crc32c_verify_blocks_dev_async(hdfs3_crc_ctx *ctx, const hdfs3_dev_block *blocks, size_t n,
                                         uint32_t bpc, int check_short_tail, uint64_t *d_result) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (n == 0) return 0;
    if (!blocks || !d_result) return fail(-EINVAL, "null argument");
    DeviceGuard g(ctx->device);
    return blocks_common(ctx, blocks, n, bpc, true, check_short_tail, reinterpret_cast<unsigned long long *>(d_result));
}

int hdfs3_crc32c_verify_blocks_dev(hdfs3_crc_ctx *ctx, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc,
                                   int check_short_tail, int64_t *bad_block, int64_t *bad_chunk) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (bad_block) *bad_block = -1;
    if (bad_chunk) *bad_chunk = -1;
    if (n == 0) return 0;
    if (!blocks) return fail(-EINVAL, "null argument");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipMemsetAsync(ctx->d_result, 0, sizeof(unsigned long long), ctx->stream));
    if (int rc = blocks_common(ctx, blocks, n, bpc, true, check_short_tail, ctx->d_result)) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->h_result, ctx->d_result, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    const unsigned long long r = *ctx->h_result;
    if (r) {
        const uint64_t key = ~r;
        if (bad_block) *bad_block = int64_t(key >> 32);
        if (bad_chunk) *bad_chunk = int64_t(key & 0xFFFFFFFFu);
    }
    return 0;
}

int hdfs3_crc32c_compute_blocks_dev(hdfs3_crc_ctx *ctx, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (n == 0) return 0;
    if (!blocks) return fail(-EINVAL, "null argument");
    DeviceGuard g(ctx->device);
    return blocks_common(ctx, blocks, n, bpc, false, 0, nullptr);
}

int hdfs3_crc_abi_version(void) { return HDFS3_CRC_ABI_VERSION; }

const char *hdfs3_crc_last_error(void) { return g_err; }

int hdfs3_device_count(int *count) {
    if (!count) return fail(-EINVAL, "null count");
    HIP_TRY(hipGetDeviceCount(count));
    return 0;
}

int hdfs3_crc_ctx_create(int device, hdfs3_crc_ctx **out) {
    if (!out) return fail(-EINVAL, "null out");
    *out = nullptr;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(-ENODEV, "device %d not present (%d visible)", device, ndev);
    hdfs3_crc_ctx *ctx = new (std::nothrow) hdfs3_crc_ctx();
    if (!ctx) return fail(-ENOMEM, "ctx allocation");
    ctx->device = device;
    DeviceGuard g(device);
    auto bail = [&](int rc) {
        hdfs3_crc_ctx_destroy(ctx);
        return rc;
    };
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return bail(fail(-EIO, "hipGetDeviceProperties(%d) failed", device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return bail(fail(-ENODEV, "device %d is %s; this build targets gfx950 (MI355X) only",
                         device, prop.gcnArchName));
    ctx->grid_cap = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(-EIO, "hipStreamCreate failed"));
    ctx->stream = ctx->own_stream;
    if (hipMalloc(reinterpret_cast<void **>(&ctx->d_result), sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&ctx->h_result), sizeof(unsigned long long),
                      hipHostMallocDefault) != hipSuccess)
        return bail(fail(-ENOMEM, "device allocation for ctx failed"));
    const HostImage *img = host_images();
    for (int p = 0; p < 2; ++p) {
        if (hipMalloc(reinterpret_cast<void **>(&ctx->d_tables_by[p]), sizeof(img[p].t)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&ctx->d_fold_by[p]), kFoldUploadBytes) != hipSuccess)
            return bail(fail(-ENOMEM, "device allocation for ctx failed"));
        if (hipMemcpy(ctx->d_tables_by[p], img[p].t, sizeof(img[p].t), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(ctx->d_fold_by[p], img[p].fold, kFoldUploadBytes, hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(-EIO, "table upload failed"));
    }
    ctx->d_tables = ctx->d_tables_by[0];
    ctx->d_fold = ctx->d_fold_by[0];
    ctx->poly = kPolyReflected;
    *out = ctx;
    return 0;
}

void hdfs3_crc_ctx_destroy(hdfs3_crc_ctx *ctx) {
    if (!ctx) return;
    DeviceGuard g(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (Slot &s : ctx->slot) {
        if (s.h_data) (void)hipHostFree(s.h_data);
        if (s.h_crc) (void)hipHostFree(s.h_crc);
        if (s.d_data) (void)hipFree(s.d_data);
        if (s.d_crc) (void)hipFree(s.d_crc);
        if (s.done) (void)hipEventDestroy(s.done);
    }
    for (PacketArena &a : ctx->arena_cache) a.release();
    ctx->arena_cache.clear();
    for (auto &st : ctx->seg_ring) {
        if (st.h) (void)hipHostFree(st.h);
        if (st.d) (void)hipFree(st.d);
        if (st.done) (void)hipEventDestroy(st.done);
        if (st.copied) (void)hipEventDestroy(st.copied);
    }
    if (ctx->desc_stream) {
        (void)hipStreamSynchronize(ctx->desc_stream);
        (void)hipStreamDestroy(ctx->desc_stream);
    }
    ctx->words.release();
    ctx->pieces.release();
    for (int p = 0; p < 2; ++p) {
        if (ctx->d_tables_by[p]) (void)hipFree(ctx->d_tables_by[p]);
        if (ctx->d_fold_by[p]) (void)hipFree(ctx->d_fold_by[p]);
    }
    if (ctx->d_result) (void)hipFree(ctx->d_result);
    if (ctx->h_result) (void)hipHostFree(ctx->h_result);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
}

}  // extern "C"

namespace hdfs3crc {
namespace {
std::mutex g_ctx_pool_mu;
std::vector<hdfs3_crc_ctx *> g_ctx_pool;
constexpr size_t kCtxPoolMax = 32;
constexpr size_t kArenaCacheKeep = 6;  // arenas any pooled ctx keeps (block_reader.cpp kArenaCacheMax)
constexpr size_t kDeepCtxMax = 8;      // pooled contexts allowed to keep a read-ahead ring's worth
// 1 GiB: the rings of a read-ahead stream up to depth 3 (whole 128 MiB blocks) plus the usual
// shallow contexts; with 512 MiB, depth 2 / 3 read 9.1-10.7 / 5.1-7.0 GiB/s against 13.2-13.9 /
// 11.1-14.1 (every open re-pinned rings the pool had shed; profiles/r03/reentry/r3e2e_caps_*)
constexpr uint64_t kPoolPinnedDefault = uint64_t(1) << 30;

// HDFS3_POOL_PINNED_MAX: bytes, or with a K/M/G suffix
uint64_t pool_pinned_cap() {
    static const uint64_t cap = [] {
        const char *e = std::getenv("HDFS3_POOL_PINNED_MAX");
        if (!e || !*e) return kPoolPinnedDefault;
        char *end = nullptr;
        const unsigned long long v = std::strtoull(e, &end, 10);
        const int shift = *end == 'K' || *end == 'k' ? 10 : *end == 'M' || *end == 'm' ? 20
                          : *end == 'G' || *end == 'g' ? 30 : 0;
        // a whole number with at most one K/M/G suffix; anything else ("1.5G", "64MiB", "-1")
        // is not silently read as a prefix of itself: the default stays and a warning says so
        const char *rest = end + (shift ? 1 : 0);
        if (end == e || *e == '-' || *rest != '\0' || (shift && v > (~0ull >> shift))) {
            std::fprintf(stderr, "libhdfs3_crc: HDFS3_POOL_PINNED_MAX=\"%s\" is not a byte count "
                                 "(digits with an optional K/M/G suffix); using the default %llu bytes\n",
                         e, (unsigned long long)kPoolPinnedDefault);
            return kPoolPinnedDefault;
        }
        return uint64_t(v) << shift;
    }();
    return cap;
}

struct Footprint {
    uint64_t pinned = 0, device = 0;
};

// what a ctx holds beyond its tables: pinned host and device bytes of its staging slots, cached
// arenas (with their piece scratch), descriptor stagings, word and piece scratch and result word
Footprint footprint(hdfs3_crc_ctx *ctx) {
    Footprint f;
    for (const Slot &s : ctx->slot) {
        f.pinned += s.data_cap + s.crc_cap;
        f.device += s.data_cap + s.crc_cap;
    }
    {
        std::lock_guard<std::mutex> lk(ctx->arena_mu);
        for (const PacketArena &a : ctx->arena_cache) {
            const uint64_t desc = a.desc_cap * sizeof(DevSegment) + (a.h_res ? sizeof(unsigned long long) : 0);
            f.pinned += a.cap + desc;
            // the arena's own piece scratch (bpc = R x 4096 batches) stays allocated while it is cached
            f.device += a.cap + desc + a.pieces.cap[0] + a.pieces.cap[1];
        }
    }
    for (const auto &st : ctx->seg_ring) {
        f.pinned += st.cap * sizeof(DevSegment);
        f.device += st.cap * sizeof(DevSegment);
    }
    f.pinned += sizeof(unsigned long long);
    f.device += ctx->words.cap + ctx->pieces.cap[0] + ctx->pieces.cap[1] + sizeof(unsigned long long);
    for (int p = 0; p < 2; ++p) f.device += sizeof(host_images()[p].t) + kFoldUploadBytes;
    return f;
}

// give back what a pooled ctx can rebuild on demand: cached arenas beyond `keep`, then the
// staging slots of the host API
void shed(hdfs3_crc_ctx *ctx, size_t keep_arenas, bool slots) {
    DeviceGuard g(ctx->device);
    {
        std::lock_guard<std::mutex> alk(ctx->arena_mu);
        while (ctx->arena_cache.size() > keep_arenas) {
            ctx->arena_cache.back().release();
            ctx->arena_cache.pop_back();
        }
    }
    if (!slots) return;
    for (Slot &s : ctx->slot) {
        if (s.h_data) (void)hipHostFree(s.h_data);
        if (s.h_crc) (void)hipHostFree(s.h_crc);
        if (s.d_data) (void)hipFree(s.d_data);
        if (s.d_crc) (void)hipFree(s.d_crc);
        s.h_data = s.h_crc = s.d_data = s.d_crc = nullptr;
        s.data_cap = s.crc_cap = 0;
    }
}
}  // namespace

uint64_t pool_pinned_cap_bytes() { return pool_pinned_cap(); }

std::mutex &pool_admission_mu() {
    static std::mutex mu;
    return mu;
}

void ctx_footprint(hdfs3_crc_ctx *ctx, uint64_t *pinned, uint64_t *device) {
    const Footprint f = footprint(ctx);
    if (pinned) *pinned = f.pinned;
    if (device) *device = f.device;
}

uint64_t ctx_pool_pinned_bytes() {
    std::lock_guard<std::mutex> lk(g_ctx_pool_mu);
    uint64_t n = 0;
    for (hdfs3_crc_ctx *c : g_ctx_pool) n += footprint(c).pinned;
    return n;
}

int ctx_acquire(int device, hdfs3_crc_ctx **out, bool deep) {
    if (!out) return fail(-EINVAL, "null out");
    {
        std::lock_guard<std::mutex> lk(g_ctx_pool_mu);
        // deep: the pooled ctx with the most cached arenas (a read-ahead reader's ring);
        // otherwise the one with the fewest, which keeps the deep ones for read-ahead
        long best = -1;
        for (size_t i = 0; i < g_ctx_pool.size(); ++i) {
            if (g_ctx_pool[i]->device != device) continue;
            if (best < 0 || (deep ? g_ctx_pool[i]->arena_cache.size() > g_ctx_pool[size_t(best)]->arena_cache.size()
                                  : g_ctx_pool[i]->arena_cache.size() < g_ctx_pool[size_t(best)]->arena_cache.size()))
                best = long(i);
        }
        if (best >= 0) {
            hdfs3_crc_ctx *ctx = g_ctx_pool[size_t(best)];
            g_ctx_pool.erase(g_ctx_pool.begin() + best);
            ctx->stream = ctx->own_stream;
            ctx->checksum_type = HDFS3_CHECKSUM_TYPE_CRC32C;
            ctx->d_tables = ctx->d_tables_by[0];
            ctx->d_fold = ctx->d_fold_by[0];
            ctx->poly = kPolyReflected;
            *out = ctx;
            return 0;
        }
    }
    return hdfs3_crc_ctx_create(device, out);
}

void ctx_release(hdfs3_crc_ctx *ctx) {
    if (!ctx) return;
    bool ok;
    {
        DeviceGuard g(ctx->device);
        ok = hipStreamSynchronize(ctx->stream) == hipSuccess;
    }
    for (Slot &s : ctx->slot) s.pending_out = nullptr;
    if (ok) {
        // one admission at a time across both pools (pool_admission_mu): the short-circuit readers'
        // pool counts against the same cap, and its bytes cannot grow while this decision is made
        std::lock_guard<std::mutex> adm(pool_admission_mu());
        const uint64_t local = local_pool_stats().pinned;
        std::lock_guard<std::mutex> lk(g_ctx_pool_mu);
        if (g_ctx_pool.size() < kCtxPoolMax) {
            // a read-ahead reader's deep ring leaves up to a block's worth of pinned arenas in
            // its ctx (block_reader.cpp); at most kDeepCtxMax pooled contexts keep that much,
            // the others go back to the usual few arenas
            size_t deep = 0;
            for (hdfs3_crc_ctx *c : g_ctx_pool) deep += c->arena_cache.size() > kArenaCacheKeep;
            if (deep >= kDeepCtxMax && ctx->arena_cache.size() > kArenaCacheKeep) shed(ctx, kArenaCacheKeep, false);
            // and the pool as a whole retains at most pool_pinned_cap() pinned bytes. The ctx released
            // last is the one most likely to be taken again soon (a read-ahead stream releases the
            // ring of the block it finished and at once acquires a deep ctx for the next block ahead),
            // so the pooled contexts give back their arenas first, least recently released first
            // (the pool's front); then this ctx sheds arenas and staging, and is destroyed if it still
            // does not fit. Shedding this ctx first made every read-ahead block re-pin its ring once
            // older pooled rings filled the cap: 1 GiB with read-ahead 2 / 7 at 6.6 / 2.3 GiB/s
            // against 11.8 / 10.6 uncapped (profiles/r03/reentry/r3e2eab_*).
            const uint64_t cap = pool_pinned_cap() > local ? pool_pinned_cap() - local : 0;
            const uint64_t mine = footprint(ctx).pinned;
            uint64_t others = 0;
            for (hdfs3_crc_ctx *c : g_ctx_pool) others += footprint(c).pinned;
            for (const bool slots : {false, true})  // their arenas first, then their staging slots
                for (size_t i = 0; i < g_ctx_pool.size() && others + mine > cap; ++i) {
                    const uint64_t before = footprint(g_ctx_pool[i]).pinned;
                    shed(g_ctx_pool[i], 0, slots);
                    others -= before - footprint(g_ctx_pool[i]).pinned;
                }
            if (others + footprint(ctx).pinned > cap) shed(ctx, 0, false);
            if (others + footprint(ctx).pinned > cap) shed(ctx, 0, true);
            if (others + footprint(ctx).pinned <= cap) {
                g_ctx_pool.push_back(ctx);
                return;
            }
        }
    }
    hdfs3_crc_ctx_destroy(ctx);
}

}  // namespace hdfs3crc

extern "C" {

int hdfs3_crc_ctx_acquire(int device, hdfs3_crc_ctx **out) { return hdfs3crc::ctx_acquire(device, out); }
void hdfs3_crc_ctx_release(hdfs3_crc_ctx *ctx) { hdfs3crc::ctx_release(ctx); }

int hdfs3_crc_pool_stats_get(hdfs3_crc_pool_stats *out) {
    if (!out) return fail(-EINVAL, "null out");
    hdfs3_crc_pool_stats st{};
    // the short-circuit readers' pooled contexts and windows are part of the same budget
    const hdfs3crc::LocalPoolStats lp = hdfs3crc::local_pool_stats();
    std::lock_guard<std::mutex> lk(hdfs3crc::g_ctx_pool_mu);
    for (hdfs3_crc_ctx *c : hdfs3crc::g_ctx_pool) {
        const hdfs3crc::Footprint f = hdfs3crc::footprint(c);
        st.pinned_bytes += f.pinned;
        st.device_bytes += f.device;
    }
    st.pinned_bytes += lp.pinned;
    st.device_bytes += lp.device;
    st.pooled_contexts = hdfs3crc::g_ctx_pool.size() + lp.entries;
    st.pinned_cap_bytes = hdfs3crc::pool_pinned_cap();
    *out = st;
    return 0;
}

int hdfs3_crc_pool_trim(void) {
    const int local = hdfs3crc::local_pool_trim();
    std::vector<hdfs3_crc_ctx *> idle;
    {
        std::lock_guard<std::mutex> lk(hdfs3crc::g_ctx_pool_mu);
        idle.swap(hdfs3crc::g_ctx_pool);
    }
    for (hdfs3_crc_ctx *c : idle) hdfs3_crc_ctx_destroy(c);
    return int(idle.size()) + local;
}

int hdfs3_crc_ctx_set_stream(hdfs3_crc_ctx *ctx, void *hip_stream) {
    if (!ctx) return fail(-EINVAL, "null ctx");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->own_stream;
    return 0;
}

void *hdfs3_crc_ctx_get_stream(hdfs3_crc_ctx *ctx) { return ctx ? ctx->stream : nullptr; }

int hdfs3_crc_ctx_set_checksum_type(hdfs3_crc_ctx *ctx, int type) {
    if (!ctx) return fail(-EINVAL, "null ctx");
    if (type != HDFS3_CHECKSUM_TYPE_CRC32C && type != HDFS3_CHECKSUM_TYPE_CRC32)
        return fail(-EINVAL, "checksum type %d has no CRC polynomial", type);
    const int i = type == HDFS3_CHECKSUM_TYPE_CRC32C ? 0 : 1;
    ctx->d_tables = ctx->d_tables_by[i];
    ctx->d_fold = ctx->d_fold_by[i];
    ctx->poly = i == 0 ? kPolyReflected : kPolyCrc32;
    ctx->checksum_type = type;
    return 0;
}

int hdfs3_crc_ctx_get_checksum_type(hdfs3_crc_ctx *ctx) { return ctx ? ctx->checksum_type : -EINVAL; }

int hdfs3_crc_ctx_synchronize(hdfs3_crc_ctx *ctx) {
    if (!ctx) return fail(-EINVAL, "null ctx");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

uint64_t hdfs3_crc_ctx_kernel_launches(hdfs3_crc_ctx *ctx) { return ctx ? ctx->launches.load() : 0; }

int64_t hdfs3_crc_decode_result(uint64_t r) { return r ? int64_t(~r) : -1; }

int hdfs3_crc32c_compute(hdfs3_crc_ctx *ctx, const void *data, size_t len, uint32_t bpc,
                         void *crc_be_out) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (len == 0) return 0;
    if (!data || !crc_be_out) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    return host_pipeline(ctx, data, len, bpc, nullptr, crc_be_out, 0, nullptr);
}

int hdfs3_crc32c_verify(hdfs3_crc_ctx *ctx, const void *data, size_t len, uint32_t bpc,
                        const void *crc_be, int check_short_tail, int64_t *first_bad_chunk) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (first_bad_chunk) *first_bad_chunk = -1;
    if (len == 0) return 0;
    if (!data || !crc_be) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    return host_pipeline(ctx, data, len, bpc, crc_be, nullptr, check_short_tail, first_bad_chunk);
}

int hdfs3_crc32c_compute_dev(hdfs3_crc_ctx *ctx, const void *d_data, size_t len, uint32_t bpc,
                             void *d_crc_be_out) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (len == 0) return 0;
    if (!d_data || !d_crc_be_out) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    ChunkLaunch a{};
    a.data = static_cast<const uint8_t *>(d_data);
    a.len = len;
    a.bpc = bpc;
    a.out_be = static_cast<uint8_t *>(d_crc_be_out);
    return launch(ctx, a, false);
}

int hdfs3_crc32c_compute_dev_async_ex(hdfs3_crc_ctx *ctx, const void *d_data, size_t len, uint32_t bpc,
                                      void *d_crc_be_out, uint32_t flags) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (flags & ~HDFS3_LAUNCH_OVERLAP_PREVIOUS) return fail(-EINVAL, "unknown launch flags 0x%x", flags);
    if (len == 0) return 0;
    if (!d_data || !d_crc_be_out) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    ChunkLaunch a{};
    a.data = static_cast<const uint8_t *>(d_data);
    a.len = len;
    a.bpc = bpc;
    a.out_be = static_cast<uint8_t *>(d_crc_be_out);
    a.overlap_previous = (flags & HDFS3_LAUNCH_OVERLAP_PREVIOUS) != 0;
    return launch(ctx, a, false);
}

int hdfs3_crc32c_verify_dev_async(hdfs3_crc_ctx *ctx, const void *d_data, size_t len,
                                  uint32_t bpc, const void *d_crc_be, int check_short_tail,
                                  uint64_t *d_result) {
    return hdfs3_crc32c_verify_dev_async_ex(ctx, d_data, len, bpc, d_crc_be, check_short_tail, d_result, 0);
}

int hdfs3_crc32c_verify_dev_async_ex(hdfs3_crc_ctx *ctx, const void *d_data, size_t len,
                                     uint32_t bpc, const void *d_crc_be, int check_short_tail,
                                     uint64_t *d_result, uint32_t flags) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (flags & ~HDFS3_LAUNCH_OVERLAP_PREVIOUS) return fail(-EINVAL, "unknown launch flags 0x%x", flags);
    if (len == 0) return 0;
    if (!d_data || !d_crc_be || !d_result) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    ChunkLaunch a{};
    a.data = static_cast<const uint8_t *>(d_data);
    a.len = len;
    a.bpc = bpc;
    a.crc_be = static_cast<const uint8_t *>(d_crc_be);
    a.result = reinterpret_cast<unsigned long long *>(d_result);
    a.check_short_tail = check_short_tail;
    a.overlap_previous = (flags & HDFS3_LAUNCH_OVERLAP_PREVIOUS) != 0;
    return launch(ctx, a, true);
}

int hdfs3_crc32c_verify_dev(hdfs3_crc_ctx *ctx, const void *d_data, size_t len, uint32_t bpc,
                            const void *d_crc_be, int check_short_tail, int64_t *first_bad_chunk) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (first_bad_chunk) *first_bad_chunk = -1;
    if (len == 0) return 0;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipMemsetAsync(ctx->d_result, 0, sizeof(unsigned long long), ctx->stream));
    if (int rc = hdfs3_crc32c_verify_dev_async(ctx, d_data, len, bpc, d_crc_be, check_short_tail,
                                               reinterpret_cast<uint64_t *>(ctx->d_result)))
        return rc;
    HIP_TRY(hipMemcpyAsync(ctx->h_result, ctx->d_result, sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (first_bad_chunk) *first_bad_chunk = hdfs3_crc_decode_result(*ctx->h_result);
    return 0;
}

int hdfs3_crc32c_verify_packets(hdfs3_crc_ctx *ctx, const void *arena, size_t arena_len,
                                const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc,
                                int check_short_tail, int64_t *bad_packet, int64_t *bad_chunk) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (bad_packet) *bad_packet = -1;
    if (bad_chunk) *bad_chunk = -1;
    if (n == 0) return 0;
    if (!arena || !pk) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    Slot &s = ctx->slot[0];
    if (s.done) HIP_TRY(hipEventSynchronize(s.done));
    if (int rc = finish_pending(s)) return rc;
    if (int rc = grow_slot(s, arena_len, 4)) return rc;
    CopyPool::get().copy(s.h_data, arena, arena_len);  // split over the pool from 2 MiB up
    HIP_TRY(hipMemcpyAsync(s.d_data, s.h_data, arena_len, hipMemcpyHostToDevice, ctx->stream));
    return packets_common(ctx, s.d_data, arena_len, pk, n, bpc, true, check_short_tail, bad_packet,
                          bad_chunk);
}

int hdfs3_crc32c_verify_packets_dev(hdfs3_crc_ctx *ctx, const void *d_arena, size_t arena_len,
                                    const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc,
                                    int check_short_tail, int64_t *bad_packet,
                                    int64_t *bad_chunk) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (bad_packet) *bad_packet = -1;
    if (bad_chunk) *bad_chunk = -1;
    if (n == 0) return 0;
    if (!d_arena || !pk) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    return packets_common(ctx, static_cast<const uint8_t *>(d_arena), arena_len, pk, n, bpc, true,
                          check_short_tail, bad_packet, bad_chunk);
}

int hdfs3_crc32c_compute_packets_dev(hdfs3_crc_ctx *ctx, void *d_arena, size_t arena_len,
                                     const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (n == 0) return 0;
    if (!d_arena || !pk) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    return packets_common(ctx, static_cast<const uint8_t *>(d_arena), arena_len, pk, n, bpc, false,
                          0, nullptr, nullptr);
}

int hdfs3_crc32c_verify_packets_dev_async(hdfs3_crc_ctx *ctx, const void *d_arena, size_t arena_len,
                                          const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc, int check_short_tail,
                                          uint64_t *d_result) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (n == 0) return 0;
    if (!d_arena || !pk || !d_result) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    return packets_async(ctx, static_cast<const uint8_t *>(d_arena), arena_len, pk, n, bpc, true, check_short_tail,
                         reinterpret_cast<unsigned long long *>(d_result), false);
}

int hdfs3_crc32c_compute_packets_dev_async(hdfs3_crc_ctx *ctx, void *d_arena, size_t arena_len,
                                           const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (n == 0) return 0;
    if (!d_arena || !pk) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    return packets_async(ctx, static_cast<const uint8_t *>(d_arena), arena_len, pk, n, bpc, false, 0, nullptr, false);
}

int hdfs3_crc32c_verify_packet_stream_dev_async(hdfs3_crc_ctx *ctx, const void *d_arena, size_t arena_len,
                                                const hdfs3_pkt_stream *ps, uint32_t bpc, int check_short_tail,
                                                uint64_t *d_result, uint32_t flags) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (flags & ~HDFS3_LAUNCH_OVERLAP_PREVIOUS) return fail(-EINVAL, "unknown launch flags 0x%x", flags);
    if (!ps) return fail(-EINVAL, "null stream");
    if (ps->n == 0) return 0;
    if (!d_arena || !d_result) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    return packet_stream_async(ctx, static_cast<const uint8_t *>(d_arena), arena_len, ps, bpc, true, check_short_tail,
                               reinterpret_cast<unsigned long long *>(d_result),
                               (flags & HDFS3_LAUNCH_OVERLAP_PREVIOUS) != 0);
}

int hdfs3_crc32c_compute_packet_stream_dev_async(hdfs3_crc_ctx *ctx, void *d_arena, size_t arena_len,
                                                 const hdfs3_pkt_stream *ps, uint32_t bpc) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (!ps) return fail(-EINVAL, "null stream");
    if (ps->n == 0) return 0;
    if (!d_arena) return fail(-EINVAL, "null buffer");
    DeviceGuard g(ctx->device);
    return packet_stream_async(ctx, static_cast<const uint8_t *>(d_arena), arena_len, ps, bpc, false, 0, nullptr,
                               false);
}

uint32_t hdfs3_crc32c_update_host(uint32_t state, const void *p, size_t len) {
    return len ? host_update(state, p, len) : state;
}

// Block checksum (include/hdfs3_crc.h): the CRC words come from the compute kernel in
// pieces of up to kMd5PieceChunks chunks, alternating between the two slots, so the host
// digests piece i while the GPU computes and copies out piece i+1.
namespace {
constexpr uint64_t kMd5PieceChunks = 1ull << 20;  // 4 MiB of CRC words per piece
}

int hdfs3_block_checksum_dev(hdfs3_crc_ctx *ctx, const void *d_data, size_t len, uint32_t bpc,
                             uint8_t *md5_out, uint64_t *crc_per_block) {
    if (int rc = check_args(ctx, bpc)) return rc;
    if (!md5_out || (len && !d_data)) return fail(-EINVAL, "null buffer");
    const uint64_t n = (uint64_t(len) + bpc - 1) / bpc;
    if (crc_per_block) *crc_per_block = n;
    Md5 md5;
    if (n) {
        DeviceGuard g(ctx->device);
        const uint64_t per = kMd5PieceChunks;
        const uint64_t pieces = (n + per - 1) / per;
        for (Slot &s : ctx->slot) {
            if (int rc = finish_pending(s)) return rc;
            if (int rc = grow_slot(s, 0, size_t(std::min(n, per)) * 4)) return rc;
            if (!s.done) HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        }
        auto issue = [&](uint64_t i) -> int {
            Slot &s = ctx->slot[i & 1];
            const uint64_t c0 = i * per, cn = std::min(per, n - c0);
            const uint64_t off = c0 * bpc;
            ChunkLaunch a{};
            a.data = static_cast<const uint8_t *>(d_data) + off;
            a.len = std::min<uint64_t>(cn * bpc, uint64_t(len) - off);
            a.bpc = bpc;
            a.out_be = s.d_crc;
            if (int rc = launch(ctx, a, false)) return rc;
            HIP_TRY(hipMemcpyAsync(s.h_crc, s.d_crc, size_t(cn) * 4, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipEventRecord(s.done, ctx->stream));
            return 0;
        };
        if (int rc = issue(0)) return rc;
        for (uint64_t i = 0; i < pieces; ++i) {
            if (i + 1 < pieces)
                if (int rc = issue(i + 1)) return rc;
            Slot &s = ctx->slot[i & 1];
            HIP_TRY(hipEventSynchronize(s.done));
            md5.update(s.h_crc, size_t(std::min(per, n - i * per)) * 4);
        }
    }
    md5.finish(md5_out);
    return 0;
}

int hdfs3_block_checksum_crcs(const void *crc_be, uint64_t n_crcs, uint8_t *md5_out) {
    if (!md5_out || (n_crcs && !crc_be)) return fail(-EINVAL, "null buffer");
    Md5 md5;
    md5.update(crc_be, size_t(n_crcs) * 4);
    md5.finish(md5_out);
    return 0;
}

int hdfs3_file_checksum_md5md5crc(const uint8_t *block_md5s, size_t n_blocks, uint8_t *md5_out) {
    if (!md5_out || (n_blocks && !block_md5s)) return fail(-EINVAL, "null buffer");
    Md5 md5;
    md5.update(block_md5s, n_blocks * 16);
    md5.finish(md5_out);
    return 0;
}

int hdfs3_dev_malloc(void **d_ptr, size_t bytes) {
    if (!d_ptr) return fail(-EINVAL, "null out");
    HIP_TRY(hipMalloc(d_ptr, bytes));
    return 0;
}

int hdfs3_dev_free(void *d_ptr) {
    HIP_TRY(hipFree(d_ptr));
    return 0;
}

int hdfs3_host_malloc_pinned(void **h_ptr, size_t bytes) {
    if (!h_ptr) return fail(-EINVAL, "null out");
    HIP_TRY(hipHostMalloc(h_ptr, bytes, hipHostMallocDefault));
    return 0;
}

int hdfs3_host_free_pinned(void *h_ptr) {
    HIP_TRY(hipHostFree(h_ptr));
    return 0;
}

int hdfs3_memcpy_h2d(hdfs3_crc_ctx *ctx, void *d_dst, const void *h_src, size_t bytes) {
    if (!ctx) return fail(-EINVAL, "null ctx");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

int hdfs3_memcpy_d2h(hdfs3_crc_ctx *ctx, void *h_dst, const void *d_src, size_t bytes) {
    if (!ctx) return fail(-EINVAL, "null ctx");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

int hdfs3_memset_dev(hdfs3_crc_ctx *ctx, void *d_dst, int value, size_t bytes) {
    if (!ctx) return fail(-EINVAL, "null ctx");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipMemsetAsync(d_dst, value, bytes, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

}  // extern "C"

// ---- measurement hooks: libhdfs3_crc_lab.so only (HDFS3_LAB=1; bench.py's read ceiling,
// tools/, the A/B tests). Not part of hdfs3_crc.h and not exported by libhdfs3_crc.so. ----
#if HDFS3_LAB
extern "C" {

// Coalesced read-only stream over [d, d+len): the achievable HBM read ceiling.
int hdfs3x_stream_read_ex(hdfs3_crc_ctx *ctx, const void *d, size_t len, int grid, void *d_sink, uint32_t flags);
int hdfs3x_stream_read(hdfs3_crc_ctx *ctx, const void *d, size_t len, int grid, void *d_sink) {
    return hdfs3x_stream_read_ex(ctx, d, len, grid, d_sink, 0);
}

// flags: HDFS3_LAUNCH_OVERLAP_PREVIOUS, for the same-shape ceiling of overlapped verifies
int hdfs3x_stream_read_ex(hdfs3_crc_ctx *ctx, const void *d, size_t len, int grid, void *d_sink, uint32_t flags) {
    if (!ctx) return fail(-EINVAL, "null ctx");
    DeviceGuard g(ctx->device);
    HIP_TRY(launch_stream_read(static_cast<const uint8_t *>(d), len, static_cast<uint32_t *>(d_sink),
                               grid != 0 ? grid : ctx->grid_cap * 8, ctx->stream,
                               (flags & HDFS3_LAUNCH_OVERLAP_PREVIOUS) != 0));
    return 0;
}

// The CRC kernel's chunk-per-lane access pattern without the table arithmetic.
int hdfs3x_lane_read(hdfs3_crc_ctx *ctx, const void *d, size_t len, uint32_t bpc, void *d_sink) {
    if (!ctx) return fail(-EINVAL, "null ctx");
    DeviceGuard g(ctx->device);
    HIP_TRY(launch_lane_read(static_cast<const uint8_t *>(d), len, bpc, static_cast<uint32_t *>(d_sink),
                             ctx->grid_cap, ctx->stream));
    return 0;
}

int hdfs3x_grid_cap(hdfs3_crc_ctx *ctx) { return ctx ? ctx->grid_cap : 0; }

// Process-wide kernel-variant knob for in-process A/B measurements (tools/ab.py).
void hdfs3x_set_variant(int v) { set_variant(v); }

// Clock stamps of variant 125 and the stream-read kernel (tools/clock_ramp.py): installs a device
// buffer of cap x 4 u64 ({s_memtime, s_memrealtime} at workgroup 0's start and end, one slot per
// launch); returns the number of stamps written into the previous buffer, or a negative errno.
int hdfs3x_clock_stamps(void *d_buf, unsigned int cap) {
    unsigned int n = 0;
    HIP_TRY(lab_clock_buffer(static_cast<unsigned long long *>(d_buf), cap, &n));
    return int(n);
}

int hdfs3x_wave_stamps(void *d_buf, unsigned int cap) {
    unsigned int n = 0;
    HIP_TRY(lab_wave_buffer(static_cast<unsigned long long *>(d_buf), cap, &n));
    return int(n);
}

}  // extern "C"
#endif  // HDFS3_LAB
