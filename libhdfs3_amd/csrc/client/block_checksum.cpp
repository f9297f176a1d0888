// OP_BLOCK_CHECKSUM client (include/hdfs3_client.h): what DataTransferProtocolSender::
// blockChecksum (DataTransferProtocolSender.cpp:169-180) leaves as a TODO in the
// reference, written against the op code it declares (DataTransferProtocolSender.h:49)
// and the messages of datatransfer.proto:128-130, 189-227. One request per connection,
// like every data-transfer op; the error messages follow the reference's style.
#include "hdfs3_client.h"

#include <cerrno>
#include <cstring>
#include <string>

#include "../ctx.h"
#include "net.h"
#include "wire.h"

using namespace hdfs3crc;

namespace {
constexpr size_t kMaxResponse = 10u << 20;  // RemoteBlockReader.cpp:116
constexpr int kDefaultTimeoutMs = 60000;
}  // namespace

int hdfs3_block_checksum_remote(const char *host, int port, const hdfs3_block_id *block, int timeout_ms,
                                hdfs3_block_checksum_info *out) {
    if (!host || !block || !out) return fail(-EINVAL, "invalid argument");
    std::memset(out, 0, sizeof(*out));
    out->crc_type = -1;
    const int to = timeout_ms > 0 ? timeout_ms : kDefaultTimeoutMs;
    wire::ExtendedBlock b;
    b.pool_id = block->pool_id ? block->pool_id : "";
    b.block_id = block->block_id;
    b.generation_stamp = block->generation_stamp;
    b.num_bytes = block->num_bytes;

    const int fd = net::connect_tcp(host, port, to);
    if (fd < 0) return fail(fd, "DataTransferProtocolSender: failed to connect to datanode %s:%d", host, port);
    const std::string frame = wire::encode_block_checksum(b);
    std::string resp;
    int rc = net::write_fully(fd, frame.data(), frame.size(), to);
    if (rc == 0) rc = net::read_delimited(fd, resp, kMaxResponse, to);
    net::close_fd(fd);
    if (rc)
        return fail(rc, "DataTransferProtocolSender cannot send checksum request to datanode %s:%d", host, port);

    wire::BlockOpResponse r;
    if (!wire::decode_block_op_response(resp.data(), resp.size(), r))
        return fail(-EPROTO, "cannot parse BlockOpResponseProto for the block checksum from %s:%d", host, port);
    if (r.status != wire::kSuccess)
        return fail(-EIO, "datanode %s:%d returned an error for the block checksum of block %llu: %s", host, port,
                    static_cast<unsigned long long>(b.block_id),
                    r.message.empty() ? "check Datanode's log" : r.message.c_str());
    if (!r.has_checksum_response)
        return fail(-EIO, "datanode %s:%d sent no OpBlockChecksumResponseProto", host, port);
    const wire::BlockChecksumResponse &c = r.checksum_response;
    if (c.md5.size() != sizeof(out->md5))
        return fail(-EPROTO, "block checksum md5 has %zu bytes, expected 16", c.md5.size());
    out->bytes_per_crc = c.bytes_per_crc;
    out->crc_per_block = c.crc_per_block;
    std::memcpy(out->md5, c.md5.data(), sizeof(out->md5));
    out->crc_type = c.crc_type;
    return 0;
}
