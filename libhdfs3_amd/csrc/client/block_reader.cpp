// hdfs3_block_reader: RemoteBlockReader (src/client/RemoteBlockReader.cpp) with the
// per-packet CPU verify replaced by batched GPU verification (include/hdfs3_client.h).
//
// Pipeline (three stages on a ring of pinned arenas, kSlots unless the input stream's block
// read-ahead asks for a deeper ring):
//   receiver thread  socket -> arena (readNextPacket, up to batch_packets packets; each
//                    packet's data region 16-byte aligned) -> async H2D + packet kernel +
//                    result D2H + event on the ctx stream -> `ready` queue
//   GPU              verifies batch i while the receiver fills batch i+1
//   caller (read)    waits for the front batch's event, copies its verified bytes out,
//                    returns the arena to the receiver
// so socket receive, verification and delivery overlap; the reference does all three in
// sequence on the caller's thread (RemoteBlockReader::read, :332-357). Delivery only ever
// comes from a batch whose verification completed.
#include "hdfs3_client.h"

#include <hip/hip_runtime.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <time.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../copy_pool.h"
#include "../ctx.h"
#include "../numa.h"
#include "block_reader.h"
#include "hdfs3_crc.h"
#include "net.h"
#include "wire.h"

using namespace hdfs3crc;

namespace {

constexpr int kDefaultBatchPackets = 64;
constexpr int kDefaultTimeoutMs = 60000;  // input.read.timeout default (SessionConfig.cpp)
constexpr size_t kMaxResponse = 10u << 20;  // RemoteBlockReader.cpp:116
constexpr int kSlots = 3;                  // receiving / verifying / delivering
constexpr int kPhases = 8;                 // hdfs3_reader_phase_ns
constexpr int kWaitPollUs = 20;            // the caller's sleep between queries of a batch's event
std::atomic<uint64_t> g_phase_ns[kPhases] = {};

uint64_t thread_cpu_ns() {
    timespec ts{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}
constexpr int kMaxSlots = 64;              // deepest ring (read-ahead of a whole block)
constexpr int32_t kMaxPacketData = 16 << 20;  // PacketReceiver.MAX_PACKET_SIZE (Hadoop)
constexpr size_t kArenaCacheMax = 6;       // arenas a ctx keeps for its next reader
// a batch arena's room per packet: the datanode's default 64 KiB packet, its 128 words at bpc 512 and
// the 16-byte alignment of its data (larger packets close a batch early; one that does not fit an
// empty arena grows it). Round 4: 80 KiB before, so a 64-packet arena pinned 5 MiB for 4.03 MiB of
// packets and a read-ahead stream's rings overran the pool's pinned cap by a ring (config 5)
constexpr size_t kPacketGuess = 64 * 1024 + 512 + 16;

struct PacketRef {
    uint64_t data_off, crc_off;  // inside the arena
    uint32_t data_len;
    uint32_t skip;               // pendingAhead (RemoteBlockReader.cpp:264-266)
    uint32_t deliver;            // bytes of this packet inside [start, end)
};

struct Batch {
    PacketArena a;
    size_t used = 0;
    std::vector<PacketRef> pk;
    bool verified = false;
    int64_t bad_pkt = -1;
    size_t dpkt = 0, doff = 0;  // delivery cursor
    // dense layout (round 5, see receive()): words of every packet back to back from offset 0, the
    // packets' data back to back from d0; chunk0[i] = packet i's first chunk in the batch
    bool dense = false, sealed = false;
    uint64_t d0 = 0, words_used = 0, data_used = 0;
    std::vector<uint64_t> chunk0;

    void reset() {
        used = 0;
        pk.clear();
        verified = false;
        bad_pkt = -1;
        dpkt = doff = 0;
        dense = sealed = false;
        d0 = words_used = data_used = 0;
        chunk0.clear();
    }
};

// Chunk sizes the contiguous round kernels take (launch_chunks): 512 ... 4096, and R x 4096 (the
// multi-round kernel / pieces + combine). Others keep the wire layout and the chunk-per-lane kernel.
bool dense_bpc(uint32_t bpc) {
    return bpc == 512 || bpc == 1024 || bpc == 2048 || bpc == 4096 || (bpc > 4096 && bpc % 4096 == 0);
}

// HDFS3_READER_LAYOUT=wire keeps every batch in the wire layout (A/B measurement knob)
bool wire_layout_forced() {
    static const bool f = [] {
        const char *e = getenv("HDFS3_READER_LAYOUT");
        return e && std::strcmp(e, "wire") == 0;
    }();
    return f;
}

uint64_t now_ns() {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now().time_since_epoch()).count());
}

struct Timer {  // adds the scope's duration to a counter
    std::atomic<uint64_t> &acc;
    uint64_t t0 = now_ns();
    explicit Timer(std::atomic<uint64_t> &a) : acc(a) {}
    ~Timer() { acc.fetch_add(now_ns() - t0, std::memory_order_relaxed); }
};

// Set on the failing thread by every HIP failure: a local GPU / pinned-memory fault, which
// another replica cannot cure (the input stream must not fail over on it).
thread_local bool t_hip_fault = false;

#if HDFS3_LAB
// fault injection (libhdfs3_crc_lab.so only, tests/test_input_readahead.py): the next n arena
// allocations of read-ahead (prefetch) readers fail as a pinned-memory shortage would
std::atomic<int> g_fail_prefetch_arenas{0};
#endif

int hip_err(hipError_t e, const char *what) {
    t_hip_fault = true;
    return fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

#define HIP_OK(expr)                                      \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_err(e_, #expr);  \
    } while (0)

int grow(PacketArena &a, size_t cap, size_t descs) {
    if (cap > a.cap) {
        if (a.h) (void)hipHostFree(a.h);
        if (a.d) (void)hipFree(a.d);
        a.h = a.d = nullptr;
        a.cap = 0;
        HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&a.h), cap, pinned_host_flags()));
        HIP_OK(hipMalloc(reinterpret_cast<void **>(&a.d), cap));
        a.cap = cap;
    }
    if (descs > a.desc_cap) {
        if (a.h_desc) (void)hipHostFree(a.h_desc);
        if (a.d_desc) (void)hipFree(a.d_desc);
        a.h_desc = a.d_desc = nullptr;
        a.desc_cap = 0;
        HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&a.h_desc), descs * sizeof(DevSegment), pinned_host_flags()));
        HIP_OK(hipMalloc(reinterpret_cast<void **>(&a.d_desc), descs * sizeof(DevSegment)));
        a.desc_cap = descs;
    }
    if (!a.d_res) {
        HIP_OK(hipMalloc(reinterpret_cast<void **>(&a.d_res), sizeof(unsigned long long)));
        HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&a.h_res), sizeof(unsigned long long), pinned_host_flags()));
        HIP_OK(hipEventCreateWithFlags(&a.done, hipEventDisableTiming | hipEventBlockingSync));
    }
    return 0;
}

}  // namespace

struct hdfs3_block_reader {
    int fd = -1;
    int timeout_ms = kDefaultTimeoutMs;
    int batch_packets = kDefaultBatchPackets;
    bool verify = true;
    hdfs3_crc_ctx *ctx = nullptr;
    bool own_ctx = true;       // false when borrowed from an input stream
    bool prefetch = false;     // opened ahead of the cursor with its own ring (slots > 0)
    wire::ExtendedBlock block;
    int64_t start = 0, end_offset = 0;
    uint32_t chunk_size = 0;
    uint32_t checksum_size = 0;
    const uint32_t *tables = nullptr;  // slice tables of the negotiated polynomial

    // receiver-thread state (touched only by the receiver once it runs)
    int64_t recv_cursor = 0;   // "cursor" as seen by readNextPacket for the next packet
    int64_t last_seqno = -1;
    bool range_done = false;   // every packet of the range (and the trailer) received
    bool trailer_ok = false;   // the trailer was the empty last packet (readTrailingEmptyPacket)
    std::atomic<bool> local_fault{false};  // the failure is this host's GPU/memory, not the replica
    bool have_pending_hdr = false;
    wire::PacketHeader pending_hdr;
    // Header read-ahead (round 6): every data packet is followed on the wire by another packet's fixed
    // 31-byte header (the next data packet's, or the empty last packet's, RemoteBlockReader.cpp:274-286),
    // so a packet's payload receive takes that header too: one receive per packet instead of two.
    // HDFS3_READER_HEADER_AHEAD=0 (measurement knob) reads each header on its own as before.
    bool header_ahead = true;
    bool have_next_raw = false;
    uint8_t next_raw[wire::kPacketHeaderSize];

    // shared between receiver and caller, under mu
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Batch> slot;   // the ring (kSlots, or deeper for a read-ahead reader)
    std::deque<int> ready;     // launched batches in order, front = delivering
    std::deque<int> free_slots;
    bool recv_done = false;    // the receiver has finished (range complete or failed)
    int recv_error = 0;
    std::string recv_msg;
    bool stop = false;
    std::thread rx;

    // caller state
    int64_t delivered = 0;
    bool sent_status = false;
    int error = 0;             // sticky failure (-errno)
    std::string error_msg;

    std::atomic<uint64_t> packets{0}, batches{0};
    // receive, alloc, launch, wait, deliver (hdfs3x_block_reader_timing), then (round 6) the receiver's
    // waits for a free slot, the caller's waits for a ready batch, the receiver thread's CPU time:
    // summed into g_phase_ns when the reader closes (hdfs3_reader_phase_ns)
    std::atomic<uint64_t> t_ns[kPhases] = {};
    // How the caller waits for a batch's verify (round 6). Default: it queries the batch's event and
    // sleeps kWaitPollUs between queries, leaving its core to the receivers and the datanode. Measured
    // on config 5 (profiles/r06): a blocking-sync hipEventSynchronize still spun inside the runtime (the
    // 8-stream callers burnt 0.165 CPU-s per GiB, 0.057 of it copying), and a busy query loop, the
    // behaviour before round 6, more. HDFS3_READER_WAIT=block / spin (measurement knobs) select those.
    enum WaitMode { kWaitPoll, kWaitBlock, kWaitSpin } wait_mode = kWaitPoll;
    // HDFS3_READER_COPY_NT=1 (measurement knob, round 6): the copy-out with streaming stores, so the
    // caller's destination lines are written without being read first (x86 with AVX2)
    bool copy_nt = false;
    // A caller whose whole range has one destination (pread: fetchBlockByteRange) passes it at open
    // (round 6; the input stream does unless HDFS3_READER_EAGER_COPY=0): the receiver copies each
    // packet's bytes there right after its receive, while they are hot in cache, and read() skips the
    // copy for output that lands where they already are. Delivery and errors are unchanged: read() still returns only verified
    // bytes; bytes past a bad packet may already sit in the caller's buffer beyond the count returned.
    uint8_t *dest = nullptr;
    int64_t rx_out = 0;  // receiver: bytes of the range copied to dest so far
    void eager(const uint8_t *src, int64_t useful) {
        if (dest && useful > 0 && rx_out + useful <= end_offset - start) std::memcpy(dest + rx_out, src, size_t(useful));
        rx_out += useful;
    }

    int sticky(int code, const std::string &msg) {
        error = code;
        error_msg = msg;
        return fail(code, "%s", msg.c_str());
    }

    // RemoteBlockReader::checkResponse (:112-203); runs on the opening thread
    int check_response() {
        std::string resp;
        if (int rc = net::read_delimited(fd, resp, kMaxResponse, timeout_ms))
            return sticky(rc, "RemoteBlockReader: failed to read BlockOpResponseProto");
        wire::BlockOpResponse r;
        if (!wire::decode_block_op_response(resp.data(), resp.size(), r))
            return sticky(-EPROTO, "RemoteBlockReader cannot parse BlockOpResponseProto from Datanode response");
        if (r.status != wire::kSuccess)
            return sticky(-EIO, "RemoteBlockReader: Datanode return an error when sending read request: " +
                                    (r.message.empty() ? std::string("check Datanode's log") : r.message));
        if (!r.has_checksum_info) return sticky(-EPROTO, "RemoteBlockReader: response lacks ReadOpChecksumInfoProto");
        chunk_size = r.bytes_per_checksum;
        switch (r.checksum_type) {
        case wire::kChecksumNull: verify = false; checksum_size = 0; break;
        case wire::kChecksumCrc32c: checksum_size = 4; tables = ctx->d_tables_by[0]; break;
        // the engine switch of :158-189 (Crc32 for CHECKSUM_CRC32): the zlib-polynomial image
        case wire::kChecksumCrc32: checksum_size = 4; tables = ctx->d_tables_by[1]; break;
        default: return sticky(-EPROTO, "RemoteBlockReader cannot recognize checksum type");
        }
        // any bytesPerChecksum > 0 (:150-156; the reference's int chunkSize rejects >= 2^31, and
        // a zero size would divide by zero in its readNextPacket, :239)
        if (chunk_size == 0 || chunk_size > 0x7FFFFFFFu)
            return sticky(-EPROTO, "RemoteBlockReader invalid chunk size");
        const int64_t first = int64_t(r.chunk_offset);
        if (first < 0 || first > start || first <= start - int64_t(chunk_size))
            return sticky(-EPROTO, "RemoteBlockReader invalid first chunk offset");
        return 0;
    }

    // ---- receiver thread --------------------------------------------------------------
    // Receiver-side failures carry their message back through recv_msg (fail() is thread-local).
    int rx_fail(int code, const std::string &msg) {
        recv_msg = msg;
        return code;
    }

    int read_header(wire::PacketHeader &h) {
        if (have_pending_hdr) {
            h = pending_hdr;
            have_pending_hdr = false;
            return 0;
        }
        if (have_next_raw) {  // received with the previous packet's payload
            have_next_raw = false;
            if (!h.decode(next_raw, sizeof(next_raw))) return rx_fail(-EPROTO, "Invalid PacketHeader");
            return 0;
        }
        uint8_t buf[wire::kPacketHeaderSize];
        if (int rc = net::recv_fully(fd, buf, sizeof(buf)))
            return rx_fail(rc, "RemoteBlockReader: failed to read block header");
        if (!h.decode(buf, sizeof(buf))) return rx_fail(-EPROTO, "Invalid PacketHeader");
        return 0;
    }

    // readNextPacket (:226-277) for up to batch_packets packets into `b`
    int receive(Batch &b) {
        Timer tm(t_ns[0]);
        b.reset();
        while (int(b.pk.size()) < batch_packets && !range_done) {
            wire::PacketHeader h;
            if (int rc = read_header(h)) return rc;
            if (!h.sanity_check(last_seqno)) return rx_fail(-EIO, "RemoteBlockReader: Packet failed on sanity check");
            if (h.data_len <= 0) {  // the empty last packet ends the block
                last_seqno = h.seqno;
                range_done = true;
                break;
            }
            // stricter than the reference on malformed input (it asserts, :237-243): a bounded
            // packet (Hadoop's PacketReceiver MAX_PACKET_SIZE) that continues the byte stream
            if (h.data_len > kMaxPacketData) return rx_fail(-EIO, "Invalid Packet, dataLen exceeds 16 MiB");
            if (h.offset_in_block > recv_cursor || recv_cursor - h.offset_in_block >= h.data_len)
                return rx_fail(-EIO, "Invalid Packet, offsetInBlock does not continue the block");
            const uint64_t chunks = (uint64_t(h.data_len) + chunk_size - 1) / chunk_size;
            const uint64_t crc_len = chunks * checksum_size;
            if (int64_t(h.packet_len) != 4 + int64_t(h.data_len) + int64_t(crc_len))
                return rx_fail(-EIO, "Invalid Packet, packetLen does not match dataLen and checksums");
            const uint64_t size = crc_len + uint64_t(h.data_len);
            if (b.pk.empty())
                b.dense = verify && checksum_size == 4 && dense_bpc(chunk_size) && !wire_layout_forced();
            if (b.dense) {
                // Dense layout (round 5): the socket's [words][data] of each packet land in two places,
                // the words after the batch's earlier words, the data after its earlier data. While every
                // packet but the last holds whole chunks, the batch is then ONE contiguous block with its
                // own .meta-style word array, and the GPU verifies it with the contiguous round kernel
                // (launch()): no packet pitch, no 4 KiB rounds straddling packets. Same bytes on the
                // wire, same delivery (PacketRef), same ChecksumException semantics.
                if (b.pk.empty()) {
                    // room for batch_packets packets' words, sized for the largest packet expected (a
                    // datanode's 64 KiB, or this one if larger): a short first packet must not
                    // shrink the word region and close the batch after a few packets
                    const uint64_t exp_data = std::max<uint64_t>(uint64_t(h.data_len), uint64_t(64) << 10);
                    const uint64_t max_crc = (exp_data + chunk_size - 1) / chunk_size * checksum_size;
                    b.d0 = (uint64_t(batch_packets) * max_crc + 4095) & ~uint64_t(4095);
                    // the arena as acquired holds the batch (64 KiB packets: 32 KiB of words + 4 MiB of
                    // data in the 64 x 66,064 B the ring is sized for); larger packets close the batch
                    // early, as in the wire layout, and only a single packet that does not fit grows it
                    const uint64_t need = b.d0 + uint64_t(h.data_len);
                    if (need > b.a.cap)
                        if (int rc = grow(b.a, need, size_t(batch_packets))) return rx_fail(rc, "arena growth failed");
                } else if (b.sealed || b.words_used + crc_len > b.d0 ||
                           b.d0 + b.data_used + uint64_t(h.data_len) > b.a.cap) {
                    pending_hdr = h;  // close this batch; the header opens the next
                    have_pending_hdr = true;
                    break;
                }
                // the packet's checksums and data in one scatter read (:244-245 reads them as one buffer)
                iovec v[3] = {{b.a.h + b.words_used, crc_len}, {b.a.h + b.d0 + b.data_used, size_t(h.data_len)},
                              {next_raw, header_ahead ? sizeof(next_raw) : 0}};
                if (int rc = net::recv_fully_iov(fd, v, 3))
                    return rx_fail(rc, "RemoteBlockReader: failed to read packet payload");
                have_next_raw = header_ahead;
                last_seqno = h.seqno;
                packets.fetch_add(1, std::memory_order_relaxed);
                int64_t ahead = recv_cursor - h.offset_in_block;
                ahead = ahead > 0 ? ahead : 0;
                const int64_t useful =
                    std::max<int64_t>(0, std::min<int64_t>(h.data_len - ahead, end_offset - recv_cursor));
                b.pk.push_back(PacketRef{b.d0 + b.data_used, b.words_used, uint32_t(h.data_len), uint32_t(ahead),
                                         uint32_t(useful)});
                eager(b.a.h + b.d0 + b.data_used + ahead, useful);
                b.chunk0.push_back(b.words_used / 4);
                b.words_used += crc_len;
                b.data_used += uint64_t(h.data_len);
                b.used = b.d0 + b.data_used;
                if (h.data_len % chunk_size) b.sealed = true;  // a short chunk ends the contiguous chunk run
                const int64_t reached = recv_cursor + h.data_len - ahead;
                recv_cursor = reached;
                if (reached >= end_offset) {
                    if (int rc = read_trailer()) return rc;
                    range_done = true;
                }
                continue;
            }
            uint64_t off = ((b.used + crc_len + 15) & ~uint64_t(15)) - crc_len;
            if (off + size > b.a.cap) {
                if (!b.pk.empty()) {  // close this batch; the header opens the next
                    pending_hdr = h;
                    have_pending_hdr = true;
                    break;
                }
                if (int rc = grow(b.a, size + 64, size_t(batch_packets))) return rx_fail(rc, "arena growth failed");
                off = ((crc_len + 15) & ~uint64_t(15)) - crc_len;
            }
            iovec v[2] = {{b.a.h + off, size}, {next_raw, header_ahead ? sizeof(next_raw) : 0}};
            if (int rc = net::recv_fully_iov(fd, v, 2))
                return rx_fail(rc, "RemoteBlockReader: failed to read packet payload");
            have_next_raw = header_ahead;
            last_seqno = h.seqno;
            packets.fetch_add(1, std::memory_order_relaxed);
            int64_t ahead = recv_cursor - h.offset_in_block;
            ahead = ahead > 0 ? ahead : 0;
            const int64_t useful = std::max<int64_t>(0, std::min<int64_t>(h.data_len - ahead, end_offset - recv_cursor));
            b.pk.push_back(PacketRef{off + crc_len, off, uint32_t(h.data_len), uint32_t(ahead), uint32_t(useful)});
            eager(b.a.h + off + crc_len + ahead, useful);
            b.used = off + size;
            const int64_t reached = recv_cursor + h.data_len - ahead;
            recv_cursor = reached;
            if (reached >= end_offset) {
                if (int rc = read_trailer()) return rc;
                range_done = true;
            }
        }
        return 0;
    }

    // readTrailingEmptyPacket (:279-287): the datanode follows the range with an empty last packet
    int read_trailer() {
        wire::PacketHeader t;
        if (int rc = read_header(t)) return rc;
        if (t.last_packet_in_block && t.data_len == 0) {
            last_seqno = t.seqno;
            trailer_ok = true;
        }
        return 0;
    }

    int launch(Batch &b) {
        Timer tm(t_ns[2]);
        batches.fetch_add(1, std::memory_order_relaxed);
        if (!verify) {
            b.verified = true;
            return 0;
        }
        const uint32_t *fold = ctx->d_fold_by[tables == ctx->d_tables_by[1]];
        HIP_OK(hipMemcpyAsync(b.a.d, b.a.h, b.used, hipMemcpyHostToDevice, ctx->stream));
        HIP_OK(hipMemsetAsync(b.a.d_res, 0, sizeof(unsigned long long), ctx->stream));
        if (b.dense) {
            // one contiguous block of b.data_used bytes and its word array: the contiguous round kernel
            // (bpc <= 4096), the multi-round kernel or pieces + combine (R x 4096, on the batch's own
            // piece scratch); keys are the batch's chunk indices (wait() maps them to packets)
            ChunkLaunch a{};
            a.data = b.a.d + b.d0;
            a.len = b.data_used;
            a.bpc = chunk_size;
            a.crc_be = b.a.d;
            a.result = b.a.d_res;
            a.check_short_tail = 0;  // verifyChecksum ignores a short chunk's mismatch (:319)
            HIP_OK(launch_chunks(a, true, tables, fold, ctx->grid_cap, ctx->stream, &b.a.pieces));
        } else {
            std::vector<DevPacket> hp(b.pk.size());
            for (size_t i = 0; i < b.pk.size(); ++i)
                hp[i] = DevPacket{b.pk[i].data_off, b.pk[i].crc_off, b.pk[i].data_len, 0};
            HIP_OK(launch_packet_batch(b.a.d, hp.data(), hp.size(), chunk_size, true, /*check_short_tail=*/0, b.a.d_res,
                                       b.a.h_desc, b.a.d_desc, tables, fold, ctx->grid_cap, ctx->stream, 0, nullptr,
                                       false, nullptr, &b.a.pieces));
        }
        ++ctx->launches;
        HIP_OK(hipMemcpyAsync(b.a.h_res, b.a.d_res, sizeof(unsigned long long), hipMemcpyDeviceToHost, ctx->stream));
        HIP_OK(hipEventRecord(b.a.done, ctx->stream));
        return 0;
    }

    // an arena for `b`: already owned, else one the ctx cached from an earlier reader, else new
    int acquire(Batch &b) {
        Timer tm(t_ns[1]);
#if HDFS3_LAB
        if (prefetch && g_fail_prefetch_arenas.load() > 0 && g_fail_prefetch_arenas.fetch_sub(1) > 0) {
            t_hip_fault = true;
            return rx_fail(fail(-ENOMEM, "injected pinned-memory shortage"), "arena allocation failed");
        }
#endif
        if (!b.a.h) {
            std::lock_guard<std::mutex> lk(ctx->arena_mu);
            if (!ctx->arena_cache.empty()) {
                b.a = ctx->arena_cache.back();
                ctx->arena_cache.pop_back();
            }
        }
        if (int rc = grow(b.a, std::max(b.a.cap, size_t(batch_packets) * kPacketGuess), size_t(batch_packets)))
            return rx_fail(rc, "arena allocation failed");
        return 0;
    }

    void receiver() {
        (void)hipSetDevice(ctx->device);
        // the socket's data lands in host memory here (RemoteBlockReader.cpp:245): on the GPU's node
        bind_thread_to_device(ctx->device);
        const uint64_t cpu0 = thread_cpu_ns();
        struct CpuAdd {  // the thread's CPU time, whichever way the loop ends
            hdfs3_block_reader *r;
            uint64_t c0;
            ~CpuAdd() { r->t_ns[7].fetch_add(thread_cpu_ns() - c0, std::memory_order_relaxed); }
        } cpu_add{this, cpu0};
        for (;;) {
            int s;
            {
                Timer idle(t_ns[5]);
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !free_slots.empty(); });
                if (stop) break;
                s = free_slots.front();
                free_slots.pop_front();
            }
            Batch &b = slot[s];
            t_hip_fault = false;
            int rc = acquire(b);
            if (!rc) rc = receive(b);
            if (!rc && !b.pk.empty()) {
                rc = launch(b);
                if (rc) recv_msg = hdfs3_crc_last_error();
            }
            if (rc && t_hip_fault) local_fault = true;
            {
                std::lock_guard<std::mutex> lk(mu);
                if (!rc && !b.pk.empty())
                    ready.push_back(s);
                else
                    free_slots.push_back(s);
                if (rc) recv_error = rc;
                if (rc || range_done) recv_done = true;
            }
            cv.notify_all();
            if (rc || range_done) break;
        }
    }

    void start_receiver() {
        for (int i = 0; i < int(slot.size()); ++i) free_slots.push_back(i);
        rx = std::thread([this] { receiver(); });
    }

    // ---- caller side ----------------------------------------------------------------------
    int wait(Batch &b) {
        if (b.verified) return 0;
        Timer tm(t_ns[3]);
        if (wait_mode == kWaitBlock) {
            HIP_OK(hipEventSynchronize(b.a.done));  // a blocking-sync event (grow())
        } else {
            for (;;) {
                const hipError_t q = hipEventQuery(b.a.done);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) HIP_OK(q);
                if (wait_mode == kWaitPoll) std::this_thread::sleep_for(std::chrono::microseconds(kWaitPollUs));
            }
        }
        const unsigned long long r = *b.a.h_res;
        if (r && b.dense) {  // the first bad chunk of the batch -> its packet
            const uint64_t chunk = ~r;
            b.bad_pkt = int64_t(std::upper_bound(b.chunk0.begin(), b.chunk0.end(), chunk) - b.chunk0.begin()) - 1;
        } else if (r) {
            b.bad_pkt = int64_t((~r) >> 32);
        }
        b.verified = true;
        return 0;
    }

    // sendStatus (:289-304), once every packet of the range verified and was handed out —
    // and only when the packet after the range was the empty last packet (:274-286): a
    // datanode that keeps streaming gets no status, as from the reference
    void maybe_send_status() {
        if (sent_status || error || !trailer_ok) return;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (!recv_done || recv_error || !ready.empty()) return;
        }
        const std::string msg = wire::encode_client_read_status(verify ? wire::kChecksumOk : wire::kSuccess);
        if (net::write_delimited(fd, msg, timeout_ms) == 0) sent_status = true;
    }

    int32_t read(uint8_t *out, int32_t len) {
        if (error) return fail(error, "%s", error_msg.c_str());
        if (len <= 0 || !out) return fail(-EINVAL, "invalid read buffer");
        int32_t total = 0;
        while (total < len) {
            int s;
            {
                Timer idle(t_ns[6]);
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !ready.empty() || recv_done; });
                if (ready.empty()) {
                    if (recv_error) {  // good batches were all delivered first
                        const int code = recv_error;
                        const std::string msg = recv_msg;
                        lk.unlock();
                        if (total) {
                            error = code;
                            error_msg = msg;
                            return total;
                        }
                        return sticky(code, msg);
                    }
                    break;  // range exhausted
                }
                s = ready.front();
            }
            Batch &b = slot[s];
            if (int rc = wait(b)) {
                local_fault = true;
                return total ? total : sticky(rc, hdfs3_crc_last_error());
            }
            const size_t limit = b.bad_pkt >= 0 ? size_t(b.bad_pkt) : b.pk.size();
            {
                Timer tm(t_ns[4]);
                // (a copy per packet on this thread: splitting a call's copies over the copy
                // pool gained nothing on a single TCP-bound stream and cost 8 concurrent
                // streams ~20 %, profiles/r02/e2e_read_copy_pool_ab.jsonl)
                while (total < len && b.dpkt < limit) {
                    const PacketRef &p = b.pk[b.dpkt];
                    const size_t avail = p.deliver - b.doff;
                    const size_t n = std::min<size_t>(avail, size_t(len - total));
                    if (dest && out + total == dest + delivered)
                        ;  // the receiver already put these bytes here
                    else if (copy_nt && n >= 4096)
                        memcpy_stream(out + total, b.a.h + p.data_off + p.skip + b.doff, n);
                    else
                        std::memcpy(out + total, b.a.h + p.data_off + p.skip + b.doff, n);
                    total += int32_t(n);
                    b.doff += n;
                    delivered += int64_t(n);
                    if (b.doff == p.deliver) {
                        ++b.dpkt;
                        b.doff = 0;
                    }
                }
            }
            if (b.dpkt == limit) {
                if (b.bad_pkt >= 0) {
                    sticky(-EIO, "ChecksumException: RemoteBlockReader: checksum not match for Block: " +
                                     std::to_string(block.block_id) + " (packet " + std::to_string(b.bad_pkt) +
                                     " of a GPU batch)");
                    return total ? total : error;
                }
                {
                    std::lock_guard<std::mutex> lk(mu);
                    ready.pop_front();
                    free_slots.push_back(s);
                }
                cv.notify_all();
            }
        }
        maybe_send_status();
        return total;
    }

    int64_t available() {
        std::lock_guard<std::mutex> lk(mu);
        int64_t a = 0;
        for (int s : ready) {
            const Batch &b = slot[s];
            if (!b.verified) continue;
            const size_t limit = b.bad_pkt >= 0 ? size_t(b.bad_pkt) : b.pk.size();
            for (size_t i = b.dpkt; i < limit; ++i) a += b.pk[i].deliver - (i == b.dpkt ? b.doff : 0);
        }
        return a;
    }

    ~hdfs3_block_reader() {
        if (rx.joinable()) {
            {
                std::lock_guard<std::mutex> lk(mu);
                stop = true;
            }
            cv.notify_all();
            if (fd >= 0) shutdown(fd, SHUT_RDWR);  // unblocks a receiver waiting on the socket
            rx.join();
        }
        if (ctx) (void)hipStreamSynchronize(ctx->stream);
        for (int i = 0; i < kPhases; ++i) g_phase_ns[i].fetch_add(t_ns[i].load(), std::memory_order_relaxed);
        // a borrowed ctx keeps up to a ring's worth of arenas for its next reader (a read-ahead
        // reader's deep ring included: the stream's next read-ahead takes them back)
        const size_t cache_max = std::max(kArenaCacheMax, slot.size());
        for (Batch &b : slot) {
            if (!b.a.h) continue;
            bool cached = false;
            if (ctx && !own_ctx) {
                std::lock_guard<std::mutex> lk(ctx->arena_mu);
                if (ctx->arena_cache.size() < cache_max) {
                    ctx->arena_cache.push_back(b.a);
                    cached = true;
                }
            }
            if (!cached) b.a.release();
            b.a = PacketArena();
        }
        if (ctx && own_ctx) ctx_release(ctx);
        net::close_fd(fd);
    }
};

namespace hdfs3crc {

bool block_reader_local_fault(const hdfs3_block_reader *r) { return r && r->local_fault.load(); }

int64_t block_reader_batch_bytes(const hdfs3_reader_opts *opts) {
    const int bp = opts && opts->batch_packets > 0 ? opts->batch_packets : kDefaultBatchPackets;
    return int64_t(bp) * 64 * 1024;  // payload of a batch of 64 KiB datanode packets
}

int64_t block_reader_arena_bytes(const hdfs3_reader_opts *opts) {
    const int bp = opts && opts->batch_packets > 0 ? opts->batch_packets : kDefaultBatchPackets;
    // what acquire()/grow() pin for one batch: the arena, its descriptor staging and result word
    return int64_t(bp) * int64_t(kPacketGuess + sizeof(DevSegment)) + int64_t(sizeof(unsigned long long));
}

int open_block_reader(const char *host, int port, const hdfs3_block_id *blk, int64_t start, int64_t len,
                      const char *client_name, const hdfs3_reader_opts *opts, hdfs3_crc_ctx *shared_ctx,
                      hdfs3_block_reader **out, int slots, uint8_t *dest) {
    if (!out || !host || !blk || start < 0 || len < 0) return fail(-EINVAL, "invalid argument");
    *out = nullptr;
    hdfs3_block_reader *r = new (std::nothrow) hdfs3_block_reader();
    if (!r) return fail(-ENOMEM, "reader allocation");
    int nslots = slots > 0 ? slots : kSlots;
    if (const char *e = getenv("HDFS3_READER_SLOTS"); e && slots <= 0)  // measurement knob (config5_ab)
        nslots = std::atoi(e);
    r->slot.resize(size_t(std::min(std::max(nslots, kSlots), kMaxSlots)));
    r->prefetch = slots > 0;
    {
        const char *w = getenv("HDFS3_READER_WAIT");
        r->wait_mode = !w                            ? hdfs3_block_reader::kWaitPoll
                       : std::strcmp(w, "spin") == 0  ? hdfs3_block_reader::kWaitSpin
                       : std::strcmp(w, "block") == 0 ? hdfs3_block_reader::kWaitBlock
                                                      : hdfs3_block_reader::kWaitPoll;
        const char *ha = getenv("HDFS3_READER_HEADER_AHEAD");
        r->header_ahead = !(ha && ha[0] == '0');
#if HDFS3_COPY_NT_AVAILABLE
        const char *nt = getenv("HDFS3_READER_COPY_NT");
        r->copy_nt = nt && nt[0] == '1' && __builtin_cpu_supports("avx2");
#endif
    }
    const int device = opts ? opts->device : 0;
    r->verify = opts ? opts->verify != 0 : true;
    if (opts && opts->batch_packets > 0) r->batch_packets = opts->batch_packets;
    if (const char *bp = getenv("HDFS3_READER_BATCH_PACKETS")) {  // measurement knob (tools/config5_ab.py)
        const int v = std::atoi(bp);
        if (v > 0 && v <= 1024) r->batch_packets = v;
    }
    if (opts && opts->timeout_ms > 0) r->timeout_ms = opts->timeout_ms;
    r->block.pool_id = blk->pool_id ? blk->pool_id : "";
    r->block.block_id = blk->block_id;
    r->block.generation_stamp = blk->generation_stamp;
    r->block.num_bytes = blk->num_bytes;
    r->start = r->recv_cursor = start;
    r->end_offset = start + len;
    r->dest = dest;
    if (shared_ctx) {
        r->ctx = shared_ctx;
        r->own_ctx = false;
    } else if (int rc = ctx_acquire(device, &r->ctx)) {
        delete r;
        return rc;
    }
    r->fd = net::connect_tcp(host, port, r->timeout_ms);
    if (r->fd < 0) {
        const int rc = r->fd;
        delete r;
        return fail(rc, "RemoteBlockReader: Failed to connect to %s:%d", host, port);
    }
    wire::ReadBlockRequest req;
    req.block = r->block;
    req.client_name = client_name ? client_name : "libhdfs3_amd";
    req.offset = uint64_t(start);
    req.len = uint64_t(len);
    const std::string frame = wire::encode_read_block(req);
    if (int rc = net::write_fully(r->fd, frame.data(), frame.size(), r->timeout_ms)) {
        delete r;
        return fail(rc, "DataTransferProtocolSender cannot send read request to datanode");
    }
    if (int rc = r->check_response()) {
        delete r;
        return rc;
    }
    // the receiver's blocking reads (net::recv_fully) time out through SO_RCVTIMEO, set once here
    if (int rc = net::set_recv_timeout(r->fd, r->timeout_ms)) {
        delete r;
        return fail(rc, "RemoteBlockReader: cannot set the socket's read timeout");
    }
    r->start_receiver();  // read-ahead starts now, as RemoteBlockReader's first read would
    *out = r;
    return 0;
}

}  // namespace hdfs3crc

extern "C" {

int hdfs3_block_reader_open(const char *host, int port, const hdfs3_block_id *blk, int64_t start,
                            int64_t len, const char *client_name, const hdfs3_reader_opts *opts,
                            hdfs3_block_reader **out) {
    return open_block_reader(host, port, blk, start, len, client_name, opts, nullptr, out);
}

int32_t hdfs3_block_reader_read(hdfs3_block_reader *r, void *buf, int32_t len) {
    if (!r) return fail(-EINVAL, "null reader");
    return r->read(static_cast<uint8_t *>(buf), len);
}

int64_t hdfs3_block_reader_available(hdfs3_block_reader *r) { return r ? r->available() : 0; }

int hdfs3_block_reader_stats(hdfs3_block_reader *r, uint32_t *bpc, uint64_t *packets, uint64_t *gpu_batches) {
    if (!r) return fail(-EINVAL, "null reader");
    if (bpc) *bpc = r->chunk_size;
    if (packets) *packets = r->packets.load();
    if (gpu_batches) *gpu_batches = r->batches.load();
    return 0;
}

#if HDFS3_LAB
void hdfs3x_fail_prefetch_arenas(int n) { g_fail_prefetch_arenas = n; }

// measurement hook (libhdfs3_crc_lab.so only): nanoseconds spent per phase so far
int hdfs3x_block_reader_timing(hdfs3_block_reader *r, uint64_t *out5) {
    if (!r || !out5) return fail(-EINVAL, "invalid argument");  // the first 5 phases
    for (int i = 0; i < 5; ++i) out5[i] = r->t_ns[i].load();
    return 0;
}
#endif

int hdfs3_block_reader_close(hdfs3_block_reader *r) {
    delete r;
    return 0;
}

int hdfs3_reader_phase_ns(uint64_t *out, int n, int reset) {
    if (!out || n < 0 || n > kPhases) return fail(-EINVAL, "invalid argument");
    for (int i = 0; i < n; ++i) out[i] = reset ? g_phase_ns[i].exchange(0) : g_phase_ns[i].load();
    if (reset)
        for (int i = n; i < kPhases; ++i) g_phase_ns[i].store(0);
    return 0;
}

}  // extern "C"
