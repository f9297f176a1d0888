// TEST / BENCH INFRASTRUCTURE — a loopback "datanode" serving in-memory blocks over the
// HDFS data-transfer protocol, so the GPU block reader can be exercised end to end
// without a cluster (the reference has no in-process datanode either: SURVEY.md §4).
// Server side of the exchange the reference client drives in RemoteBlockReader.cpp:
//   request  BE16 version | u8 op | varint len | OpReadBlockProto
//   response varint len | BlockOpResponseProto {SUCCESS, ChecksumProto, chunkOffset}
//   packets  [31 B PacketHeader][chunks x BE32 CRC][data] ..., then an empty last packet
//   status   varint len | ClientReadStatusProto (CHECKSUM_OK / SUCCESS) from the client
// CRC words are served as given (the caller computes them; corrupt ones for negative
// tests). Data and CRC buffers are referenced, not copied.
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <sys/socket.h>
#include <sys/uio.h>
#include <thread>
#include <unistd.h>

#include "../../libhdfs3_amd/csrc/client/net.h"
#include "../../libhdfs3_amd/csrc/client/wire.h"

using namespace hdfs3crc;

namespace {

struct Block {
    const uint8_t *data;
    uint64_t len;
    const uint8_t *crc_be;  // ceil(len/bpc) words
    uint32_t bpc;
    int type;
};

std::mutex g_mu;
std::map<uint64_t, Block> g_blocks;
std::atomic<int> g_listen_fd{-1};
std::atomic<bool> g_stop{false};
std::atomic<int> g_packet_bytes{64 * 1024};
std::atomic<uint64_t> g_served{0};
std::atomic<int> g_last_status{-1};
std::thread g_accept;

int send_all_iov(int fd, iovec *iov, int n) {
    size_t total = 0;
    for (int i = 0; i < n; ++i) total += iov[i].iov_len;
    while (total) {
        msghdr m{};
        m.msg_iov = iov;
        m.msg_iovlen = size_t(n);
        // MSG_NOSIGNAL: a client that stops early (ChecksumException) must not SIGPIPE the host
        ssize_t w = sendmsg(fd, &m, MSG_NOSIGNAL);
        if (w < 0) {
            if (errno == EINTR || errno == EAGAIN) continue;
            return -errno;
        }
        total -= size_t(w);
        while (n && size_t(w) >= iov->iov_len) {
            w -= ssize_t(iov->iov_len);
            ++iov;
            --n;
        }
        if (n) {
            iov->iov_base = static_cast<char *>(iov->iov_base) + w;
            iov->iov_len -= size_t(w);
        }
    }
    return 0;
}

void serve(int fd) {
    const int to = 60000;
    uint8_t head[3];
    std::string proto;
    wire::ReadBlockRequest req;
    if (net::read_fully(fd, head, 3, to) || net::read_delimited(fd, proto, 1 << 20, to) ||
        !wire::decode_read_block(proto.data(), proto.size(), req)) {
        net::close_fd(fd);
        return;
    }
    wire::BlockOpResponse resp;
    Block b{};
    bool found = false;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_blocks.find(req.block.block_id);
        if (it != g_blocks.end()) b = it->second, found = true;
    }
    const int version = (head[0] << 8) | head[1];
    if (version != wire::kDataTransferVersion || head[2] != wire::kOpReadBlock || !found ||
        req.offset > b.len) {
        resp.status = wire::kErrorInvalid;
        resp.message = found ? "bad request" : "block not found";
        net::write_delimited(fd, wire::encode_block_op_response(resp), to);
        net::close_fd(fd);
        return;
    }
    const uint64_t first = req.offset - req.offset % b.bpc;  // reads align back to a chunk
    uint64_t end = req.offset + req.len;
    if (end > b.len) end = b.len;
    resp.status = wire::kSuccess;
    resp.has_checksum_info = true;
    resp.checksum_type = b.type;
    resp.bytes_per_checksum = b.bpc;
    resp.chunk_offset = first;
    if (net::write_delimited(fd, wire::encode_block_op_response(resp), to)) {
        net::close_fd(fd);
        return;
    }
    const uint64_t per = std::max<uint64_t>(b.bpc, uint64_t(g_packet_bytes.load()) / b.bpc * b.bpc);
    const uint32_t csize = b.type == wire::kChecksumNull ? 0 : 4;
    int64_t seq = 0;
    for (uint64_t pos = first; pos < end; pos += per) {
        uint64_t n = end - pos < per ? end - pos : per;
        n = std::min<uint64_t>(((n + b.bpc - 1) / b.bpc) * b.bpc, b.len - pos);  // whole chunks
        const uint64_t chunks = (n + b.bpc - 1) / b.bpc;
        wire::PacketHeader h;
        h.packet_len = int32_t(4 + n + chunks * csize);
        h.offset_in_block = int64_t(pos);
        h.seqno = seq++;
        h.last_packet_in_block = false;
        h.data_len = int32_t(n);
        uint8_t hb[wire::kPacketHeaderSize];
        h.encode(hb);
        iovec iov[3] = {{hb, sizeof(hb)},
                        {const_cast<uint8_t *>(b.crc_be + 4 * (pos / b.bpc)), size_t(chunks * csize)},
                        {const_cast<uint8_t *>(b.data + pos), size_t(n)}};
        if (send_all_iov(fd, iov, 3)) {
            net::close_fd(fd);
            return;
        }
        g_served += n;
        if (pos + n >= end) break;
    }
    wire::PacketHeader last;
    last.packet_len = 4;
    last.offset_in_block = int64_t(end);
    last.seqno = seq;
    last.last_packet_in_block = true;
    last.data_len = 0;
    uint8_t lb[wire::kPacketHeaderSize];
    last.encode(lb);
    if (net::write_fully(fd, lb, sizeof(lb), to) == 0) {
        std::string st;
        int status = -1;
        if (net::read_delimited(fd, st, 1024, 10000) == 0 &&
            wire::decode_client_read_status(st.data(), st.size(), status))
            g_last_status = status;
    }
    net::close_fd(fd);
}

void accept_loop() {
    for (;;) {
        const int lfd = g_listen_fd.load();
        if (lfd < 0 || g_stop) return;
        const int fd = accept(lfd, nullptr, nullptr);
        if (fd < 0) {
            if (g_stop) return;
            continue;
        }
        std::thread(serve, fd).detach();
    }
}

}  // namespace

extern "C" {

int hdfs3_loopback_start(int *port) {
    if (g_listen_fd >= 0) return -EBUSY;
    int p = 0;
    const int fd = net::listen_tcp(0, &p);
    if (fd < 0) return fd;
    g_stop = false;
    g_listen_fd = fd;
    g_accept = std::thread(accept_loop);
    if (port) *port = p;
    return 0;
}

int hdfs3_loopback_add_block(uint64_t block_id, const void *data, uint64_t len, const void *crc_be,
                             uint32_t bpc, int checksum_type) {
    if (!bpc) return -EINVAL;
    std::lock_guard<std::mutex> lk(g_mu);
    g_blocks[block_id] = Block{static_cast<const uint8_t *>(data), len, static_cast<const uint8_t *>(crc_be), bpc,
                               checksum_type};
    return 0;
}

void hdfs3_loopback_clear_blocks(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_blocks.clear();
}

void hdfs3_loopback_set_packet_bytes(int n) { g_packet_bytes = n > 0 ? n : 64 * 1024; }
uint64_t hdfs3_loopback_served_bytes(void) { return g_served.load(); }
int hdfs3_loopback_last_status(void) { return g_last_status.load(); }

int hdfs3_loopback_stop(void) {
    const int fd = g_listen_fd.exchange(-1);
    g_stop = true;
    if (fd >= 0) {
        shutdown(fd, SHUT_RDWR);
        net::close_fd(fd);
    }
    if (g_accept.joinable()) g_accept.join();
    return 0;
}

}  // extern "C"
