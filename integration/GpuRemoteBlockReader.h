/*
 * GpuRemoteBlockReader — libhdfs3's BlockReader interface (src/client/BlockReader.h:36-61)
 * over hdfs3_block_reader (include/hdfs3_client.h): the RemoteBlockReader of
 * src/client/RemoteBlockReader.cpp with its per-packet CPU verify (:306-326) replaced by
 * read-ahead batches verified on the GPU. A mismatch surfaces as ChecksumException
 * (src/common/Exception.h:116-125), so InputStreamImpl::readOneBlock's replica failover
 * (InputStreamImpl.cpp:682-704) keeps working unchanged; transport and protocol errors are
 * HdfsIOException, as in the reference.
 *
 * Where it plugs in: InputStreamImpl::setupBlockReader (InputStreamImpl.cpp:418-421),
 * instead of `new RemoteBlockReader(...)`, with the block's pool id / id / generation
 * stamp / length and the datanode's transfer address:
 *     blockReader = shared_ptr<BlockReader>(new GpuRemoteBlockReader(
 *         dn.getIpAddr().c_str(), dn.getXferPort(), b.getPoolId().c_str(), b.getBlockId(),
 *         b.getGenerationStamp(), b.getNumBytes(), offset, len, clientName.c_str(), verify,
 *         conf->getGpuChecksumDevice(), conf->getInputReadTimeout()));
 *
 * Header-only; compiled against the reference's own BlockReader.h and Exception.h by
 * tests/test_reference_headers.py. The HdfsException constructors are defined in the
 * reference's Exception.cpp, so a program using this header links against libhdfs3.
 */
#ifndef HDFS3_INTEGRATION_GPUREMOTEBLOCKREADER_H
#define HDFS3_INTEGRATION_GPUREMOTEBLOCKREADER_H

#include <cerrno>
#include <cstring>
#include <string>
#include <vector>

#include "BlockReader.h"  /* src/client/BlockReader.h */
#include "Exception.h"    /* src/common/Exception.h   */
#include "hdfs3_client.h"
#include "hdfs3_crc.h"

namespace Hdfs {
namespace Internal {

class GpuRemoteBlockReader : public BlockReader {
public:
    GpuRemoteBlockReader(const char *host, int xfer_port, const char *pool_id, int64_t block_id,
                         int64_t generation_stamp, int64_t num_bytes, int64_t start, int64_t len,
                         const char *client_name, bool verify, int device, int timeout_ms) {
        hdfs3_block_id id{pool_id, static_cast<uint64_t>(block_id), static_cast<uint64_t>(generation_stamp),
                          static_cast<uint64_t>(num_bytes)};
        hdfs3_reader_opts o{device, verify ? 1 : 0, 64, timeout_ms};
        if (hdfs3_block_reader_open(host, xfer_port, &id, start, len, client_name, &o, &r) != 0)
            raise(-EIO);
    }

    ~GpuRemoteBlockReader() override { hdfs3_block_reader_close(r); }

    int64_t available() override { return hdfs3_block_reader_available(r); }

    /* RemoteBlockReader::read (:332-357): verified bytes only; a read past the end of the
     * range throws HdfsIOException (:335-338), as the reference does (callers stop on
     * available()/their own cursor, InputStreamImpl.cpp:616-708) */
    int32_t read(char *buf, int32_t size) override {
        const int32_t n = hdfs3_block_reader_read(r, buf, size);
        if (n < 0) raise(n);
        if (n == 0)
            throw HdfsIOException("RemoteBlockReader: read over block end from Datanode", __FILE__, __LINE__, "");
        return n;
    }

    /* RemoteBlockReader::skip (:359-387): read and drop, so skipped bytes are verified too */
    void skip(int64_t len) override {
        std::vector<char> scratch(len < (1 << 20) ? static_cast<size_t>(len > 0 ? len : 0) : size_t(1) << 20);
        while (len > 0) {
            const int32_t want = static_cast<int32_t>(len < int64_t(scratch.size()) ? len : int64_t(scratch.size()));
            len -= read(scratch.data(), want);
        }
    }

private:
    [[noreturn]] void raise(int rc) {
        const char *msg = hdfs3_crc_last_error();
        if (rc == -EIO && std::strstr(msg, "ChecksumException"))
            throw ChecksumException(msg, __FILE__, __LINE__, "");
        throw HdfsIOException(msg, __FILE__, __LINE__, "");
    }

    hdfs3_block_reader *r = nullptr;
};

}  // namespace Internal
}  // namespace Hdfs

#endif /* HDFS3_INTEGRATION_GPUREMOTEBLOCKREADER_H */
