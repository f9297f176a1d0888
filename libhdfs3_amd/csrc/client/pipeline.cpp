// hdfs3_pipeline: PipelineImpl (src/client/Pipeline.cpp) for the blocks of one file — the
// write-side transport behind hdfs3_output_*'s packet sink. Single-threaded like the
// reference: packets are written on the caller's thread and acks are consumed there too,
// one non-blocking check after every send (checkResponse(false), :742-753), blocking once
// more than max_unacked packets are outstanding (:631-633, waitForAcks(false)) and at
// flush / block close (waitForAcks(true), :755-813, :823-841).
//
// Per block: connect to the first node, OP_WRITE_BLOCK {PIPELINE_SETUP_CREATE (or, for the
// appended last block of hdfs3_pipeline_open_append, PIPELINE_SETUP_APPEND with the block's length
// and the new generation stamp), the other nodes as targets, ChecksumProto{type, bpc}} and the
// BlockOpResponseProto check
// (createBlockOutputStream, :529-608); then [31 B header][BE32 CRC words][data] packets
// exactly as the output stream built them (their CRCs computed on the GPU), each acked by a
// PipelineAckProto carrying one status per node (processAck, :680-722).
//
// Not rebuilt (outside the checksum path, docs/DESIGN_HISTORY.md §8): pipeline recovery
// (buildForAppendOrRecovery / resend, :610-619, a namenode RPC round), heartbeat packets and
// block tokens. A failure is therefore sticky: the stream fails with -EIO and the message the
// reference would have thrown before it started recovery.
#include <cerrno>
#include <cinttypes>
#include <cstring>
#include <deque>
#include <new>
#include <string>
#include <vector>

#include "../ctx.h"
#include "hdfs3_client.h"
#include "hdfs3_crc.h"
#include "net.h"
#include "wire.h"

using namespace hdfs3crc;

namespace {

constexpr int kDefaultTimeoutMs = 60000;
constexpr int kDefaultMaxUnacked = 1024;   // output.packetpool.size (SessionConfig.cpp:126)
constexpr size_t kMaxAck = 1 << 16;

struct BlockTarget {
    wire::ExtendedBlock id;
    std::vector<std::pair<std::string, int>> nodes;  // pipeline order
    int64_t acked = 0;                               // lastBlock->setNumBytes(bytesAcked)
    bool append = false;        // PIPELINE_SETUP_APPEND: the file's last block, `base` bytes long
    int64_t base = 0;
    uint64_t new_gs = 0;        // updateBlockForPipeline's generation stamp
};

struct Outstanding {
    int64_t seqno;
    int64_t last_byte;   // Packet::getLastByteOffsetBlock
    bool last;
};

std::string block_name(const wire::ExtendedBlock &b) {
    char buf[160];
    snprintf(buf, sizeof(buf), "[block pool ID: %s block ID %" PRIu64 "_%" PRIu64 "]", b.pool_id.c_str(), b.block_id,
             b.generation_stamp);
    return buf;
}

}  // namespace

struct hdfs3_pipeline {
    std::vector<BlockTarget> blocks;
    std::string client_name;
    uint32_t bpc = 512;
    int checksum_type = wire::kChecksumCrc32c;
    int timeout_ms = kDefaultTimeoutMs;
    int max_unacked = kDefaultMaxUnacked;

    int fd = -1;
    int64_t cur = -1;                 // block index of the open pipeline
    std::deque<Outstanding> pending;  // PipelineImpl::packets
    int64_t bytes_sent = 0, bytes_acked = 0;
    uint64_t packets = 0, acks = 0;
    int error = 0;
    std::string error_msg;

    ~hdfs3_pipeline() { net::close_fd(fd); }

    int sticky(int code, const std::string &msg) {
        if (!error) {
            error = code;
            error_msg = msg;
        }
        net::close_fd(fd);
        fd = -1;
        return fail(error, "%s", error_msg.c_str());
    }

    std::string node_name(size_t i) const {
        const auto &n = blocks[size_t(cur)].nodes[i];
        return n.first + ":" + std::to_string(n.second);
    }

    // createBlockOutputStream (:529-608) for block b: stage PIPELINE_SETUP_CREATE for a new block,
    // PIPELINE_SETUP_APPEND for the appended last block (buildForAppendOrRecovery, :214-335)
    int setup(int64_t b) {
        if (b < 0 || b >= int64_t(blocks.size()))
            return sticky(-EIO, "Pipeline: no block allocated for block " + std::to_string(b) +
                                    " of the file (addBlock returned " + std::to_string(blocks.size()) + ")");
        cur = b;
        BlockTarget &t = blocks[size_t(b)];
        bytes_sent = bytes_acked = t.append ? t.base : 0;  // PipelineImpl(bytesSent = offsetInBlock)
        const int s = net::connect_tcp(t.nodes[0].first.c_str(), t.nodes[0].second, timeout_ms);
        if (s < 0)
            return sticky(-EIO, "Cannot create block output stream for block " + block_name(t.id) +
                                    ": connect to " + node_name(0) + " failed: " + std::strerror(-s));
        fd = s;
        wire::WriteBlockRequest req;
        req.block = t.id;
        req.block.num_bytes = t.append ? uint64_t(t.base) : 0;  // lastBlock->getNumBytes()
        req.client_name = client_name;
        for (size_t i = 1; i < t.nodes.size(); ++i) {
            // BuildNodeInfo (DataTransferProtocolSender.cpp:80-90) from the namenode's DatanodeInfo; an
            // hdfs3_datanode carries the transfer address only, so the uuid, info/ipc ports and the rack
            // (location, field 8) go out empty/zero: the bytes equal the reference's for a node whose
            // namenode record has no rack (the codec itself is pinned with racks, tests/test_wire_protobuf.py)
            wire::DatanodeAddr d;
            d.ip_addr = d.host_name = t.nodes[i].first;
            d.xfer_port = uint32_t(t.nodes[i].second);
            req.targets.push_back(d);
        }
        req.stage = t.append ? wire::kPipelineSetupAppend : wire::kPipelineSetupCreate;
        if (t.append) {  // writeBlock(..., lastBlock->getNumBytes(), bytesSent, gs, ...) (:545-547)
            req.min_bytes_rcvd = uint64_t(t.base);
            req.max_bytes_rcvd = uint64_t(bytes_sent);
            req.latest_generation_stamp = t.new_gs;
        }
        req.pipeline_size = uint32_t(req.targets.size());
        req.checksum_type = checksum_type;
        req.bytes_per_checksum = bpc;
        const std::string msg = wire::encode_write_block(req);
        std::string resp_bytes;
        int rc = net::write_fully(fd, msg.data(), msg.size(), timeout_ms);
        if (!rc) rc = net::read_delimited(fd, resp_bytes, 1 << 20, timeout_ms);
        if (rc)
            return sticky(-EIO, "Cannot create block output stream for block " + block_name(t.id) +
                                    ": datanode " + node_name(0) + ": " + std::strerror(-rc));
        wire::BlockOpResponse resp;
        if (!wire::decode_block_op_response(resp_bytes.data(), resp_bytes.size(), resp))
            return sticky(-EIO, "cannot parse datanode response from " + node_name(0) + " for block " +
                                    block_name(t.id) + ".");
        if (resp.status != wire::kSuccess)
            return sticky(-EIO, "Bad connect ack with firstBadLink as " + resp.first_bad_link + " for block " +
                                    block_name(t.id));
        if (t.append) t.id.generation_stamp = t.new_gs;  // lastBlock = lb (:327-334)
        return 0;
    }

    // processResponse + processAck (:680-740)
    int process_response() {
        std::string buf;
        const BlockTarget &t = blocks[size_t(cur)];
        if (int rc = net::read_delimited(fd, buf, kMaxAck, timeout_ms))
            return sticky(-EIO, "Pipeline: failed to read the ack for block " + block_name(t.id) + " from " +
                                    node_name(0) + ": " + std::strerror(-rc));
        wire::PipelineAck ack;
        if (!wire::decode_pipeline_ack(buf.data(), buf.size(), ack))
            return sticky(-EIO, "processAllAcks: get an invalid DataStreamer packet ack for block " + block_name(t.id));
        if (ack.seqno == wire::kHeartbeatSeqno) return 0;
        ++acks;
        if (pending.empty())
            return sticky(-EIO, "processAck: unexpected ack with seqno " + std::to_string(ack.seqno) + " for block " +
                                    block_name(t.id) + ".");
        if (!ack.success()) {
            for (int i = int(ack.status.size()) - 1; i >= 0; --i)
                if (ack.status[size_t(i)] != wire::kSuccess)
                    return sticky(-EIO, "processAck: ack report error at node: " +
                                            (size_t(i) < t.nodes.size() ? node_name(size_t(i)) : std::to_string(i)) +
                                            " for block " + block_name(t.id) + ".");
        }
        const Outstanding &p = pending.front();
        if (p.seqno != ack.seqno)
            return sticky(-EIO, "processAck: pipeline ack expecting seqno " + std::to_string(p.seqno) +
                                    "  but received " + std::to_string(ack.seqno) + " for block " + block_name(t.id) +
                                    ".");
        if (p.last_byte > bytes_acked) bytes_acked = p.last_byte;
        blocks[size_t(cur)].acked = bytes_acked;
        const bool last = p.last;
        pending.pop_front();
        if (last) {  // the block is complete on every node
            net::close_fd(fd);
            fd = -1;
        }
        return 0;
    }

    // checkResponse (:742-753)
    int check_response(bool wait) {
        const int r = net::readable(fd, wait ? timeout_ms : 0);
        if (r < 0) return sticky(-EIO, std::string("Pipeline: poll failed: ") + std::strerror(-r));
        if (r > 0) return process_response();
        if (wait)
            return sticky(-EIO, "Timeout when reading response for block " + block_name(blocks[size_t(cur)].id) +
                                    ", datanode " + node_name(0) + " do not response.");
        return 0;
    }

    // waitForAcks (:759-813), without the recovery branch
    int wait_for_acks(bool force) {
        while (!pending.empty()) {
            if (!force && int(pending.size()) < max_unacked) return 0;
            if (int rc = check_response(true)) return rc;
        }
        return 0;
    }

    // PipelineImpl::send (:621-678), and close (:823-841) for the block's last packet
    int send(const void *pkt, size_t len, const hdfs3_packet_info *info) {
        if (error) return fail(error, "%s", error_msg.c_str());
        if (fd < 0 || info->block_index != cur) {
            if (fd >= 0 && !pending.empty())
                return sticky(-EIO, "Pipeline: block " + std::to_string(info->block_index) + " started before block " +
                                        std::to_string(cur) + " was closed by its last packet");
            net::close_fd(fd);
            fd = -1;
            if (int rc = setup(info->block_index)) return rc;
        }
        if (info->last_packet_in_block)
            if (int rc = wait_for_acks(true)) return rc;
        pending.push_back(Outstanding{info->seqno, info->offset_in_block + info->data_len,
                                      info->last_packet_in_block != 0});
        if (int(pending.size()) > max_unacked)
            if (int rc = wait_for_acks(false)) return rc;
        if (int rc = net::write_fully(fd, pkt, len, timeout_ms))
            return sticky(-EIO, "Pipeline: failed to send packet " + std::to_string(info->seqno) + " of block " +
                                    block_name(blocks[size_t(cur)].id) + " to " + node_name(0) + ": " +
                                    std::strerror(-rc));
        ++packets;
        const int64_t last_byte = info->offset_in_block + info->data_len;
        if (last_byte > bytes_sent) bytes_sent = last_byte;
        if (info->last_packet_in_block) return wait_for_acks(true);
        return check_response(false);
    }
};

namespace hdfs3crc {
uint32_t pipeline_bpc(const hdfs3_pipeline *p) { return p->bpc; }
}  // namespace hdfs3crc

extern "C" {

int hdfs3_pipeline_open(const hdfs3_located_block *blocks, int n_blocks, const char *client_name,
                        uint32_t bytes_per_checksum, const hdfs3_pipeline_opts *opts, hdfs3_pipeline **out) {
    if (!out || !blocks || n_blocks <= 0 || !bytes_per_checksum) return fail(-EINVAL, "invalid argument");
    *out = nullptr;
    hdfs3_pipeline *p = new (std::nothrow) hdfs3_pipeline();
    if (!p) return fail(-ENOMEM, "pipeline allocation");
    p->client_name = client_name ? client_name : "";
    p->bpc = bytes_per_checksum;
    if (opts) {
        if (opts->timeout_ms > 0) p->timeout_ms = opts->timeout_ms;
        if (opts->max_unacked > 0) p->max_unacked = opts->max_unacked;
        if (opts->checksum_type != 0) {
            if (opts->checksum_type != wire::kChecksumCrc32c) {
                delete p;
                return fail(-EINVAL, "Pipeline: the output stream computes CRC32C words only");
            }
        }
    }
    for (int i = 0; i < n_blocks; ++i) {
        const hdfs3_located_block &lb = blocks[i];
        if (!lb.replicas || lb.n_replicas <= 0 || !lb.block.pool_id) {
            delete p;
            return fail(-EINVAL, "Pipeline: block %d has no pipeline nodes", i);
        }
        BlockTarget t;
        t.id.pool_id = lb.block.pool_id;
        t.id.block_id = lb.block.block_id;
        t.id.generation_stamp = lb.block.generation_stamp;
        for (int r = 0; r < lb.n_replicas; ++r) {
            if (!lb.replicas[r].host) {
                delete p;
                return fail(-EINVAL, "Pipeline: block %d node %d has no host", i, r);
            }
            t.nodes.emplace_back(lb.replicas[r].host, lb.replicas[r].port);
        }
        p->blocks.push_back(std::move(t));
    }
    *out = p;
    return 0;
}

int hdfs3_pipeline_open_append(const hdfs3_located_block *blocks, int n_blocks, uint64_t new_generation_stamp,
                               const char *client_name, uint32_t bytes_per_checksum,
                               const hdfs3_pipeline_opts *opts, hdfs3_pipeline **out) {
    if (blocks && n_blocks > 0 && new_generation_stamp <= blocks[0].block.generation_stamp)
        return fail(-EINVAL, "Pipeline: the new generation stamp must be above the last block's");
    if (int rc = hdfs3_pipeline_open(blocks, n_blocks, client_name, bytes_per_checksum, opts, out)) return rc;
    BlockTarget &t = (*out)->blocks[0];
    t.append = true;
    t.base = int64_t(blocks[0].block.num_bytes);
    t.acked = t.base;
    t.new_gs = new_generation_stamp;
    return 0;
}

int hdfs3_pipeline_generation_stamp(hdfs3_pipeline *p, int block, uint64_t *gs) {
    if (!p || !gs || block < 0 || block >= int(p->blocks.size())) return fail(-EINVAL, "invalid argument");
    *gs = p->blocks[size_t(block)].id.generation_stamp;
    return 0;
}

int hdfs3_pipeline_send(void *pipeline, const void *packet, size_t len, const hdfs3_packet_info *info) {
    hdfs3_pipeline *p = static_cast<hdfs3_pipeline *>(pipeline);
    if (!p || !packet || !info) return fail(-EINVAL, "invalid argument");
    return p->send(packet, len, info);
}

int hdfs3_pipeline_flush(hdfs3_pipeline *p) {
    if (!p) return fail(-EINVAL, "invalid argument");
    if (p->error) return fail(p->error, "%s", p->error_msg.c_str());
    if (p->fd < 0) return 0;
    return p->wait_for_acks(true);
}

int hdfs3_pipeline_stats(hdfs3_pipeline *p, int64_t *block_bytes_acked, int n_blocks, uint64_t *packets,
                         uint64_t *acks) {
    if (!p) return fail(-EINVAL, "invalid argument");
    for (int i = 0; block_bytes_acked && i < n_blocks && i < int(p->blocks.size()); ++i)
        block_bytes_acked[i] = p->blocks[size_t(i)].acked;
    if (packets) *packets = p->packets;
    if (acks) *acks = p->acks;
    return 0;
}

const char *hdfs3_pipeline_error(hdfs3_pipeline *p) { return p && p->error ? p->error_msg.c_str() : ""; }

int hdfs3_pipeline_close(hdfs3_pipeline *p) {
    if (!p) return fail(-EINVAL, "invalid argument");
    int rc = p->error;
    if (!rc && p->fd >= 0) rc = p->wait_for_acks(true);
    delete p;
    return rc;
}

}  // extern "C"
