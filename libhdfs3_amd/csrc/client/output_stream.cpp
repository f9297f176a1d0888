// hdfs3_output_stream: OutputStreamImpl's append/flush/sync/close (src/client/
// OutputStreamImpl.cpp:298-441, 512-575) building the same wire packets as Packet
// (src/client/Packet.cpp:44-153), with the per-chunk CRC computed on the GPU in batches
// instead of Checksum::update per chunk on the caller's thread.
//
// Batch arena (pinned host, mirrored in HBM), batch_packets packet slots of
//   [lead: room for the 31 B header + chunksPerPacket BE32 words][data, 16 B aligned]
// followed by one compact CRC region (4 B per chunk of the batch). Appends copy user
// bytes straight into the current slot's data region (the reference memcpys them into
// its Packet buffer too). A full batch is dispatched: H2D of the data span, the packet
// compute kernel writing every chunk's CRC (short tail chunks included) into the compact
// region, D2H of that region, an event. Two batches alternate, so the caller fills one
// while the GPU computes the other. When a batch completes, each packet's words are
// copied in front of its data, its header in front of those, and the contiguous packet
// [header][words][data] — byte-identical to Packet::getBuffer — goes to the sink in order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../ctx.h"
#include "hdfs3_client.h"
#include "hdfs3_crc.h"
#include "wire.h"

using namespace hdfs3crc;

namespace hdfs3crc {
uint32_t pipeline_bpc(const hdfs3_pipeline *p);  // client/pipeline.cpp
}

namespace {

constexpr int kDefaultBatchPackets = 64;
constexpr int kMaxBatchPackets = 1024;
constexpr int kHeader = wire::kPacketHeaderSize;  // 31

uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

struct Pkt {
    uint64_t data_off;        // inside the arena
    int64_t offset_in_block;
    int64_t seqno;
    int64_t block_index;
    uint32_t data_len = 0;
    bool last = false;        // lastPacketInBlock (always empty)
};

struct WBatch {
    PacketArena a;
    std::vector<Pkt> pk;
    uint64_t chunks = 0;      // CRC words of the dispatched packets
    bool dispatched = false;
};

int hip_err(hipError_t e, const char *what) {
    return fail(e == hipErrorOutOfMemory ? -ENOMEM : -EIO, "%s: %s", what, hipGetErrorString(e));
}

#define HIP_OK(expr)                                      \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_err(e_, #expr);  \
    } while (0)

// hdfs.h convention: errno + -1, the message where hdfs3_crc_last_error reads it
int posix_fail(int err, const std::string &msg) {
    fail(-err, "%s", msg.c_str());
    errno = err;
    return -1;
}

}  // namespace

struct hdfs3_output_stream {
    hdfs3_crc_ctx *ctx = nullptr;
    hdfs3_packet_sink sink = nullptr;
    void *user = nullptr;
    hdfs3_pipeline *pipeline = nullptr;  // set by hdfs3_output_open_pipeline: flushed at flush/sync
    uint32_t bpc = 512;
    int32_t packet_size = 64 * 1024;
    int64_t block_size = 64ll << 20;
    int chunks_per_packet = 0;
    int batch_packets = kDefaultBatchPackets;
    uint64_t lead = 0, stride = 0, crc_region = 0, arena_bytes = 0;

    // OutputStreamImpl state
    int64_t cursor = 0, last_flushed = 0, bytes_written = 0, next_seqno = 0, block_index = 0;
    uint32_t position = 0;           // bytes of the current partial chunk
    // initAppend (OutputStreamImpl.cpp:172-230): until the first packet has been sent full, the
    // chunk size (chunkSize = freeInCksum when the file ends mid-chunk) and chunks per packet
    // (1 then, or what the last block's free space allows) differ from the configured ones
    bool is_append = false;
    uint32_t chunk_cur = 512;        // chunkSize (buffer.size())
    int cpp_cur = 0;                 // chunksPerPacket
    std::vector<uint8_t> carry;      // a flushed partial chunk, re-sent by the next packet
    bool pipeline_open = false;      // a packet of the current block has been sent
    int error = 0;
    std::string error_msg;

    WBatch batch[2];
    int cur_batch = 0;
    Pkt *cur = nullptr;              // packet being filled (last slot of batch[cur_batch])
    uint64_t packets = 0, batches = 0;

    ~hdfs3_output_stream() {
        if (ctx) {
            (void)hipStreamSynchronize(ctx->stream);
            for (WBatch &b : batch) b.a.release();
            ctx_release(ctx);
        }
    }

    int sticky(int code, const std::string &msg) {
        error = code;
        error_msg = msg;
        return fail(code, "%s", msg.c_str());
    }

    int init() {
        // computePacketChunkSize (OutputStreamImpl.cpp:161-170)
        const int with_sum = int(bpc) + 4;
        chunks_per_packet = std::max(1, (packet_size - kHeader + with_sum - 1) / with_sum);
        packet_size = chunks_per_packet * with_sum + kHeader;
        lead = align16(uint64_t(kHeader) + 4ull * chunks_per_packet);
        stride = lead + align16(uint64_t(chunks_per_packet) * bpc);
        crc_region = stride * uint64_t(batch_packets);
        arena_bytes = crc_region + 4ull * chunks_per_packet * batch_packets;
        carry.resize(bpc);
        chunk_cur = bpc;
        cpp_cur = chunks_per_packet;
        for (WBatch &b : batch) {
            HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&b.a.h), arena_bytes, hipHostMallocDefault));
            HIP_OK(hipMalloc(reinterpret_cast<void **>(&b.a.d), arena_bytes));
            b.a.cap = arena_bytes;
            HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&b.a.h_desc), batch_packets * sizeof(DevSegment),
                                 hipHostMallocDefault));
            HIP_OK(hipMalloc(reinterpret_cast<void **>(&b.a.d_desc), batch_packets * sizeof(DevSegment)));
            b.a.desc_cap = size_t(batch_packets);
            HIP_OK(hipEventCreateWithFlags(&b.a.done, hipEventDisableTiming));
            b.pk.reserve(size_t(batch_packets));
        }
        return 0;
    }

    // ---- batches ----------------------------------------------------------------------------
    int dispatch(WBatch &b) {
        if (b.dispatched || b.pk.empty()) return 0;
        b.dispatched = true;
        ++batches;
        size_t n = 0;
        uint64_t chunks = 0, lo = UINT64_MAX, hi = 0;
        DevPacket hp[kMaxBatchPackets];
        for (const Pkt &p : b.pk) {
            if (!p.data_len) continue;
            hp[n++] = DevPacket{p.data_off, crc_region + 4 * chunks, p.data_len, 0};
            chunks += (p.data_len + bpc - 1) / bpc;
            lo = std::min(lo, p.data_off);
            hi = std::max(hi, p.data_off + p.data_len);
        }
        b.chunks = chunks;
        if (n) {
            HIP_OK(hipMemcpyAsync(b.a.d + lo, b.a.h + lo, hi - lo, hipMemcpyHostToDevice, ctx->stream));
            // the batch's own piece scratch (bpc = R x 4096 batches of whole-round packets: pieces + combine)
            HIP_OK(launch_packet_batch(b.a.d, hp, n, bpc, false, 0, nullptr, b.a.h_desc, b.a.d_desc, ctx->d_tables,
                                       ctx->d_fold, ctx->grid_cap, ctx->stream, 0, nullptr, false, nullptr,
                                       &b.a.pieces));
            ++ctx->launches;
            HIP_OK(hipMemcpyAsync(b.a.h + crc_region, b.a.d + crc_region, 4 * chunks, hipMemcpyDeviceToHost,
                                  ctx->stream));
        }
        HIP_OK(hipEventRecord(b.a.done, ctx->stream));
        return 0;
    }

    // Packet::getBuffer for every packet of a completed batch, handed to the sink in order
    int emit(WBatch &b) {
        if (!b.dispatched) return 0;
        HIP_OK(hipEventSynchronize(b.a.done));
        const uint8_t *words = b.a.h + crc_region;
        for (const Pkt &p : b.pk) {
            const uint32_t nch = (p.data_len + bpc - 1) / bpc;
            uint8_t *sums = b.a.h + p.data_off - 4ull * nch;
            std::memcpy(sums, words, 4ull * nch);  // already big-endian (Packet::addChecksum)
            words += 4ull * nch;
            wire::PacketHeader h;
            h.packet_len = int32_t(p.data_len + 4 * nch + 4);  // "the server will reduce 4 bytes"
            h.offset_in_block = p.offset_in_block;
            h.seqno = p.seqno;
            h.last_packet_in_block = p.last;
            h.data_len = int32_t(p.data_len);
            uint8_t *pkt = sums - kHeader;
            h.encode(pkt);
            hdfs3_packet_info info{p.seqno, p.offset_in_block, p.block_index, int32_t(p.data_len), int32_t(nch),
                                   p.last ? 1 : 0};
            ++packets;
            if (!error) {
                const int rc = sink(user, pkt, size_t(kHeader) + 4ull * nch + p.data_len, &info);
                if (rc)
                    sticky(rc < 0 ? rc : -EIO, pipeline ? std::string(hdfs3_pipeline_error(pipeline))
                                                        : "Pipeline: the packet sink failed (seqno " +
                                                              std::to_string(p.seqno) + ")");
            }
        }
        b.pk.clear();
        b.dispatched = false;
        return error;
    }

    // a fresh packet slot; when the current batch is full it is dispatched and the other
    // batch (emitted first) becomes current
    int new_slot(Pkt **out) {
        WBatch *b = &batch[cur_batch];
        if (int(b->pk.size()) == batch_packets) {
            if (int rc = dispatch(*b)) return rc;
            cur_batch ^= 1;
            b = &batch[cur_batch];
            if (int rc = emit(*b)) return rc;
        }
        b->pk.push_back(Pkt{lead + stride * b->pk.size(), 0, 0, 0, 0, false});
        *out = &b->pk.back();
        return 0;
    }

    // packets.getPacket(packetSize, chunksPerPacket, bytesWritten, nextSeqNo++, ...)
    int open_packet() {
        Pkt *p = nullptr;
        if (int rc = new_slot(&p)) return rc;
        p->offset_in_block = bytes_written;
        p->seqno = next_seqno++;
        p->block_index = block_index;
        if (position) {  // the flushed partial chunk opens the new packet again
            std::memcpy(batch[cur_batch].a.h + p->data_off, carry.data(), position);
            p->data_len = position;
        }
        cur = p;
        return 0;
    }

    // sendPacket: the packet is complete; it leaves with its batch
    void send_current() {
        pipeline_open = true;
        if (position && cur) std::memcpy(carry.data(), batch[cur_batch].a.h + cur->data_off + cur->data_len - position,
                                         position);
        cur = nullptr;
    }

    // closePipeline (:512-536): the empty lastPacketInBlock packet at offset bytesWritten
    int close_block() {
        if (!pipeline_open) return 0;
        if (cur) send_current();
        Pkt *p = nullptr;
        if (int rc = new_slot(&p)) return rc;
        p->offset_in_block = bytes_written;
        p->seqno = next_seqno++;
        p->block_index = block_index;
        p->last = true;
        pipeline_open = false;
        bytes_written = 0;
        ++block_index;
        return 0;
    }

    // pipeline->flush(): every packet so far has reached the sink
    int drain() {
        WBatch &a = batch[cur_batch ^ 1], &b = batch[cur_batch];
        if (int rc = emit(a)) return rc;  // dispatched earlier, so it goes first
        if (int rc = dispatch(b)) return rc;
        return emit(b);
    }

    // appendInternal (:298-346)
    int append(const uint8_t *buf, int64_t size) {
        int64_t todo = size;
        while (todo > 0) {
            if (!cur)
                if (int rc = open_packet()) return rc;
            // the chunks of one packet are contiguous in its data region, so everything up to the
            // packet's or the block's end is one copy; appendChunkToPacket's per-chunk
            // bookkeeping (bytesWritten advances by whole chunks, position is the partial one)
            // is then applied for all the chunks it completed
            const uint32_t cs = chunk_cur;
            const int64_t pkt_room = int64_t(cpp_cur) * cs - cur->data_len;
            const int64_t blk_room = block_size - bytes_written - position;
            const uint32_t n = uint32_t(std::min({todo, pkt_room, blk_room}));
            std::memcpy(batch[cur_batch].a.h + cur->data_off + cur->data_len, buf + (size - todo), n);
            cur->data_len += n;
            todo -= n;
            bytes_written += int64_t((position + n) / cs) * cs;
            position = (position + n) % cs;
            const bool full = cur->data_len == uint32_t(cpp_cur) * cs;
            if (full || bytes_written == block_size) {
                send_current();
                if (is_append) {  // back to the configured chunk and packet sizes (:332-337)
                    is_append = false;
                    chunk_cur = bpc;
                    cpp_cur = chunks_per_packet;
                }
                if (bytes_written == block_size)
                    if (int rc = close_block()) return rc;
            }
        }
        cursor += size;
        return 0;
    }

    // initAppend (:172-230) for a file of file_length bytes whose last block holds last_block_bytes
    // (< 0: append() returned no last block, the next write starts a new block). The appended
    // block's packets start at offsetInBlock = last_block_bytes; a file ending mid-chunk gets a
    // first packet of ONE chunk of chunkSize - file_length % chunkSize bytes, its CRC over those
    // bytes only (the datanode merges it with the partial chunk it holds).
    int init_append(int64_t file_length, int64_t last_block_bytes) {
        cursor = last_flushed = file_length;
        if (last_block_bytes < 0) return 0;
        // The reference takes blockSize from the file's FileStatus, so bytesWritten < blockSize
        // and the last block holds file_length % blockSize bytes by construction. Here both come
        // from the caller: a block size that disagrees with the file's would make the block's
        // remaining room negative (and the copy length wrap), so it is refused up front.
        const int64_t free_in_block = block_size - file_length % block_size;
        if (free_in_block == block_size)
            return fail(-EIO, "OutputStreamImpl: the last block for the file is full.");
        if (last_block_bytes >= block_size || last_block_bytes != file_length % block_size)
            return fail(-EINVAL, "OutputStreamImpl: the last block's length does not match the file "
                                 "length and block size.");
        is_append = true;
        bytes_written = last_block_bytes;
        const uint32_t used_in_cksum = uint32_t(file_length % bpc);
        int64_t psize = packet_size;
        if (used_in_cksum > 0) {
            psize = 0;
            chunk_cur = bpc - used_in_cksum;
        } else {
            psize = std::min<int64_t>(psize, free_in_block);
        }
        // computePacketChunkSize (:161-170), C++ division truncating toward zero
        const int64_t with_sum = int64_t(chunk_cur) + 4;
        cpp_cur = int(std::max<int64_t>(1, (psize - kHeader + with_sum - 1) / with_sum));
        return 0;
    }

    // flushInternal (:392-431)
    int flush(bool need_sync) {
        if (last_flushed == cursor && !need_sync) return 0;
        last_flushed = cursor;
        if (position > 0 && !cur)
            if (int rc = open_packet()) return rc;  // re-append the buffered partial chunk
        if (!cur && need_sync && pipeline_open)
            if (int rc = open_packet()) return rc;  // an empty packet carries the sync
        if (cur) send_current();
        if (int rc = drain()) return rc;
        if (pipeline && hdfs3_pipeline_flush(pipeline))  // pipeline->flush() (:438-440)
            return sticky(-EIO, hdfs3_pipeline_error(pipeline));
        return 0;
    }

    // close (:538-575)
    int close() {
        if (!error) {
            if (last_flushed != cursor && position > 0 && !cur)
                if (int rc = open_packet()) return rc;
            if (last_flushed != cursor && cur) send_current();
            if (int rc = close_block()) return rc;
            return drain();
        }
        return error;
    }
};

extern "C" {

int hdfs3_output_open_pipeline(const hdfs3_writer_opts *opts, hdfs3_pipeline *pipeline,
                               hdfs3_output_stream **out) {
    return hdfs3_output_open_pipeline_append(opts, nullptr, pipeline, out);
}

int hdfs3_output_open_pipeline_append(const hdfs3_writer_opts *opts, const hdfs3_append_info *append,
                                      hdfs3_pipeline *pipeline, hdfs3_output_stream **out) {
    if (!pipeline || !out) return fail(-EINVAL, "invalid argument");
    const uint32_t bpc = opts && opts->bytes_per_checksum ? opts->bytes_per_checksum : 512;
    if (bpc != pipeline_bpc(pipeline))
        return fail(-EINVAL, "the pipeline's bytes per checksum differ from the stream's");
    if (int rc = hdfs3_output_open_append(opts, append, hdfs3_pipeline_send, pipeline, out)) return rc;
    (*out)->pipeline = pipeline;
    return 0;
}

int hdfs3_output_open(const hdfs3_writer_opts *opts, hdfs3_packet_sink sink, void *user,
                      hdfs3_output_stream **out) {
    return hdfs3_output_open_append(opts, nullptr, sink, user, out);
}

int hdfs3_output_open_append(const hdfs3_writer_opts *opts, const hdfs3_append_info *append, hdfs3_packet_sink sink,
                             void *user, hdfs3_output_stream **out) {
    if (!out || !sink) return fail(-EINVAL, "invalid argument");
    *out = nullptr;
    if (append && (append->file_length < 0 || append->last_block_bytes > append->file_length))
        return fail(-EINVAL, "invalid append position");
    hdfs3_output_stream *s = new (std::nothrow) hdfs3_output_stream();
    if (!s) return fail(-ENOMEM, "output stream allocation");
    s->sink = sink;
    s->user = user;
    int device = 0;
    if (opts) {
        device = opts->device;
        if (opts->bytes_per_checksum) s->bpc = opts->bytes_per_checksum;
        if (opts->packet_size > 0) s->packet_size = opts->packet_size;
        if (opts->block_size > 0) s->block_size = opts->block_size;
        if (opts->batch_packets > 0) s->batch_packets = std::min(opts->batch_packets, kMaxBatchPackets);
    }
    // OutputStreamImpl::open checks (OutputStreamImpl.cpp:258-273)
    if (s->bpc == 0 || s->packet_size < int32_t(s->bpc) || s->block_size % s->bpc != 0) {
        delete s;
        return fail(-EINVAL, "invalid packet size / chunk size / block size combination");
    }
    if (int rc = ctx_acquire(device, &s->ctx)) {
        delete s;
        return rc;
    }
    // arenas, events and launches belong to the ctx's device, whatever is current here
    DeviceGuard g(device);
    int rc = s->init();
    if (!rc && append) rc = s->init_append(append->file_length, append->last_block_bytes);
    if (rc) {
        delete s;
        return rc;
    }
    *out = s;
    return 0;
}

int32_t hdfs3_output_write(hdfs3_output_stream *s, const void *buf, int32_t len) {
    if (!s || !buf || len <= 0) return posix_fail(EINVAL, "hdfsWrite: invalid argument");
    if (s->error) return posix_fail(EIO, s->error_msg);
    DeviceGuard g(s->ctx->device);
    if (int rc = s->append(static_cast<const uint8_t *>(buf), len))
        return posix_fail(-rc, s->error ? s->error_msg : std::string(hdfs3_crc_last_error()));
    return len;
}

int hdfs3_output_flush(hdfs3_output_stream *s) {
    if (!s) return posix_fail(EINVAL, "hdfsFlush: invalid argument");
    if (s->error) return posix_fail(EIO, s->error_msg);
    DeviceGuard g(s->ctx->device);
    if (int rc = s->flush(false)) return posix_fail(-rc, s->error ? s->error_msg : hdfs3_crc_last_error());
    return 0;
}

int hdfs3_output_sync(hdfs3_output_stream *s) {
    if (!s) return posix_fail(EINVAL, "hdfsSync: invalid argument");
    if (s->error) return posix_fail(EIO, s->error_msg);
    DeviceGuard g(s->ctx->device);
    if (int rc = s->flush(true)) return posix_fail(-rc, s->error ? s->error_msg : hdfs3_crc_last_error());
    return 0;
}

int64_t hdfs3_output_tell(hdfs3_output_stream *s) {
    if (!s) return posix_fail(EINVAL, "hdfsTell: invalid argument");
    return s->cursor;
}

int hdfs3_output_stats(hdfs3_output_stream *s, uint64_t *packets, uint64_t *gpu_batches) {
    if (!s) return fail(-EINVAL, "null stream");
    if (packets) *packets = s->packets;
    if (gpu_batches) *gpu_batches = s->batches;
    return 0;
}

int hdfs3_output_close(hdfs3_output_stream *s) {
    if (!s) return posix_fail(EINVAL, "hdfsCloseFile: invalid argument");
    DeviceGuard g(s->ctx->device);  // held through the destructor's frees too
    const int rc = s->close();
    const std::string msg = s->error ? s->error_msg : (rc ? std::string(hdfs3_crc_last_error()) : std::string());
    delete s;
    if (rc) return posix_fail(-rc, msg);
    return 0;
}

}  // extern "C"
