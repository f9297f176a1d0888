/*
 * hdfs3_client.h — the block-reader surface of the drop-in (read path).
 *
 * hdfs3_block_reader is a RemoteBlockReader (src/client/RemoteBlockReader.{h,cpp})
 * whose per-packet CPU verify loop (RemoteBlockReader.cpp:306-326) is replaced by
 * batched GPU verification:
 *   - it speaks the same data-transfer protocol to a datanode: OP_READ_BLOCK framing
 *     (DataTransferProtocolSender.cpp:42-57,107-123), BlockOpResponseProto with the
 *     ChecksumProto (RemoteBlockReader.cpp:112-203), packets of
 *     [31 B header][chunks x BE32 CRC][data] (:226-277), the trailing empty packet and
 *     the final ClientReadStatusProto CHECKSUM_OK (:279-304);
 *   - packets are read ahead into a pinned arena (up to batch_packets per batch, two
 *     batches in flight) and verified on the GPU while the next batch is received;
 *   - no byte of a packet reaches the caller before its batch verified, the same
 *     invariant as the reference (verify at :253-255 precedes the memcpy at :346);
 *   - a mismatch on a full chunk returns -EIO with "ChecksumException" in
 *     hdfs3_crc_last_error(); packets before the bad one are delivered first, exactly
 *     what the reference's per-packet verify delivers before it throws. A mismatch on
 *     a short tail chunk is ignored (:319).
 * InputStreamImpl::setupBlockReader (InputStreamImpl.cpp:364-450) is where libhdfs3
 * would construct it instead of RemoteBlockReader.
 */
#ifndef HDFS3_CLIENT_H
#define HDFS3_CLIENT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hdfs3_block_reader hdfs3_block_reader;

/* ExtendedBlockProto (hdfs.proto:38-44) */
typedef struct hdfs3_block_id {
    const char *pool_id;
    uint64_t block_id;
    uint64_t generation_stamp;
    uint64_t num_bytes;
} hdfs3_block_id;

typedef struct hdfs3_reader_opts {
    int device;         /* GPU used for verification                                    */
    int verify;         /* 0: no verification (InputStream verify=false, Hdfs.cpp:722)  */
    int batch_packets;  /* packets per GPU batch (default 64 = 4 MiB at 64 KiB packets)  */
    int timeout_ms;     /* socket read/write timeout (input.read.timeout analogue)       */
} hdfs3_reader_opts;

/* Connect, send OP_READ_BLOCK for [start, start+len) and check the response
 * (RemoteBlockReader ctor, :46-75). 0 or -errno. */
int hdfs3_block_reader_open(const char *host, int port, const hdfs3_block_id *block, int64_t start,
                            int64_t len, const char *client_name, const hdfs3_reader_opts *opts,
                            hdfs3_block_reader **out);
/* RemoteBlockReader::read (:332-357): copies up to len verified bytes; returns the
 * count (> 0), 0 once the range is exhausted, or -errno (-EIO on ChecksumException). */
int32_t hdfs3_block_reader_read(hdfs3_block_reader *r, void *buf, int32_t len);
/* bytes already verified and buffered (BlockReader::available) */
int64_t hdfs3_block_reader_available(hdfs3_block_reader *r);
/* chunk size negotiated with the datanode, packets and GPU batches so far */
int hdfs3_block_reader_stats(hdfs3_block_reader *r, uint32_t *bytes_per_checksum,
                             uint64_t *packets, uint64_t *gpu_batches);
int hdfs3_block_reader_close(hdfs3_block_reader *r);

#ifdef __cplusplus
}
#endif
#endif /* HDFS3_CLIENT_H */
