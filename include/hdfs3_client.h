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
 * (RemoteBlockReader ctor, :46-75). 0 or -errno.
 * Packets are read ahead into pinned batch arenas and verified on the GPU a batch at a time. A
 * batch lands densely (every packet's checksums back to back, their data back to back) and is
 * verified as one contiguous block while its packets hold whole chunks; HDFS3_READER_LAYOUT=wire
 * keeps each packet's [checksums][data] together instead (read once per process). Delivery and
 * errors are the same either way. */
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
/* Diagnostics (round 6): nanoseconds summed over every block reader of the process that has closed
 * since the last reset, n <= 8 values in this order: the receiver's socket reads, arena acquisition,
 * launches, the caller's waits for GPU verify results, the caller's copies out, the receiver's waits
 * for a free slot (the caller is behind), the caller's waits for a received batch (the receiver is
 * behind), and the receiver threads' CPU time. reset != 0 zeroes the sums after reading them. */
int hdfs3_reader_phase_ns(uint64_t *out, int n, int reset);

/* ------------------------------------------------------------------------------------
 * Input stream: the hdfsRead / hdfsPread / hdfsSeek / hdfsTell / hdfsAvailable surface
 * (Hdfs.cpp:788-862, 924-941) over InputStreamImpl's block walk and replica failover
 * (InputStreamImpl.cpp:322-450, 583-815, 1120-1160), reading every block through
 * hdfs3_block_reader. The namenode lookup (getBlockLocations) is outside the checksum
 * path: the caller passes the LocatedBlocks it would have received.
 *
 * Error convention of these five calls is hdfs.h's, not the -errno of the rest of this
 * header, so they drop in behind hdfsRead & co unchanged: -1 with errno set
 *   EIO       every replica failed (ChecksumException or I/O) — the reference's
 *             HdfsIOException "all nodes have been tried" (InputStreamImpl.cpp:369-383)
 *   EOVERFLOW seek past the end of file (HdfsEndOfStream, Hdfs.cpp:276-277)
 *   EINVAL    bad arguments (PARAMETER_ASSERT)
 * and the message in hdfs3_crc_last_error(). read returns 0 at end of file.
 * ---------------------------------------------------------------------------------- */
typedef struct hdfs3_input_stream hdfs3_input_stream;

/* A datanode as the namenode's LocatedBlock names it, reduced to its transfer address: write
 * targets (OP_WRITE_BLOCK, DataTransferProtocolSender.cpp:80-90) go out with this host and port and
 * an empty uuid, zero info/ipc ports and an EMPTY location (rack) — the reference sends the
 * namenode's rack there (e.g. "/default-rack"); datanodes use it for nothing on this path. */
typedef struct hdfs3_datanode {  /* DatanodeInfo transfer address */
    const char *host;
    int port;
} hdfs3_datanode;

typedef struct hdfs3_located_block {  /* LocatedBlockProto (hdfs.proto) */
    hdfs3_block_id block;             /* block.num_bytes = bytes of the block in the file */
    int64_t offset;                   /* file offset of the block's first byte            */
    const hdfs3_datanode *replicas;   /* in the namenode's preference order               */
    int n_replicas;
} hdfs3_located_block;

/* Blocks must be in file order and contiguous (offset[i+1] = offset[i] + num_bytes[i]);
 * the table and host strings are copied. One GPU context per stream, taken from the process-wide
 * pool (hdfs3_crc_ctx_acquire) and returned on close. 0 or -errno. */
int hdfs3_input_open(const hdfs3_located_block *blocks, int n_blocks, const char *client_name,
                     const hdfs3_reader_opts *opts, hdfs3_input_stream **out);
/* hdfsRead: up to len bytes from the cursor, never crossing a block boundary (readOneBlock) */
int32_t hdfs3_input_read(hdfs3_input_stream *s, void *buf, int32_t len);
/* hdfsPread: reads [pos, pos+len) clipped to the file, across blocks; cursor unchanged.
 * pos outside the file returns -1 (preadInternal, InputStreamImpl.cpp:815-830). */
int32_t hdfs3_input_pread(hdfs3_input_stream *s, int64_t pos, void *buf, int32_t len);
/* hdfsSeek: a forward seek of <= 128 KiB inside the current block skips through the open
 * reader (InputStreamImpl.cpp:1146-1152); anything else reopens at the target. */
int hdfs3_input_seek(hdfs3_input_stream *s, int64_t pos);
int64_t hdfs3_input_tell(hdfs3_input_stream *s);
int hdfs3_input_available(hdfs3_input_stream *s);
int64_t hdfs3_input_length(hdfs3_input_stream *s);
/* replica failovers and block readers opened so far (diagnostics) */
int hdfs3_input_stats(hdfs3_input_stream *s, uint64_t *failovers, uint64_t *readers_opened);
/* Block read-ahead (opt-in; not in the reference, which reads one block at a time): while
 * hdfs3_input_read consumes block i, blocks i+1 .. i+blocks are read by background threads,
 * each over its own connection and pooled GPU context, verified exactly as on demand, into
 * host buffers of up to max_bytes_per_block (0 = the whole block). read() still returns the
 * same bytes, at most to the block end per call; a prefetch that hit a ChecksumException or
 * I/O error hands back the bytes it verified and the stream fails that replica over from
 * there (readOneBlock). pread is unaffected. blocks = 0 turns it off. 0 or -errno. */
#define HDFS3_READAHEAD_MAX_BLOCKS 8  /* -EINVAL above: each holds a ctx, a socket and a pinned ring */
int hdfs3_input_set_readahead(hdfs3_input_stream *s, int blocks, int64_t max_bytes_per_block);
/* block readers the read-ahead threads opened so far, and those dropped on a local (GPU or pinned
 * memory) fault, whose block was then read again on demand on the stream's own context
 * (diagnostics) */
int hdfs3_input_readahead_stats(hdfs3_input_stream *s, uint64_t *prefetch_readers_opened,
                                uint64_t *prefetch_local_faults);
int hdfs3_input_close(hdfs3_input_stream *s);

/* ------------------------------------------------------------------------------------
 * Local (short-circuit) block reader: LocalBlockReader (LocalBlockReader.cpp:46-263) over
 * a block file and its .meta file (BE16 version 1 | u8 type | BE32 bytesPerChecksum |
 * BE32 CRC per chunk). Every chunk is verified on the GPU, the short tail included
 * (:138-163); windows of window_buffers x buffer_size bytes are read ahead by a loader
 * thread. On a mismatch nothing of the buffer_size buffer holding the first bad chunk is
 * returned — the reference verifies a whole buffer before returning any of it — and
 * read returns -EIO ("ChecksumException"). Same -errno convention as the block reader.
 * ---------------------------------------------------------------------------------- */
typedef struct hdfs3_local_reader hdfs3_local_reader;

typedef struct hdfs3_local_opts {
    int device;
    int verify;               /* 0: no verification                                     */
    int32_t buffer_size;      /* input.localread.default.buffersize (1 MiB), chunk-rounded;
                                 at most 1 GiB (-EINVAL above)                           */
    int window_buffers;       /* buffers per GPU window (4)                             */
    uint32_t flags;           /* 0, or HDFS3_LOCAL_CRC32_AS_ZLIB                        */
} hdfs3_local_opts;

/* By default a .meta of type CHECKSUM_CRC32 is verified with CRC32C, exactly as the
 * reference does (both types select its CRC32C engine, LocalBlockReader.cpp:85-98), so such
 * a block fails with ChecksumException (-EIO) in both. With this flag it is verified with
 * the zlib polynomial the meta declares instead (an opt-in departure from the reference). */
#define HDFS3_LOCAL_CRC32_AS_ZLIB 1u

/* num_bytes <= 0 takes the block file's size; offset skips like LocalBlockReader::skip.
 * -EIO on a bad version or unknown type; -EINVAL on unknown flags. */
int hdfs3_local_reader_open(const char *data_path, const char *meta_path, int64_t num_bytes, int64_t offset,
                            const hdfs3_local_opts *opts, hdfs3_local_reader **out);
int32_t hdfs3_local_reader_read(hdfs3_local_reader *r, void *buf, int32_t len);
int64_t hdfs3_local_reader_available(hdfs3_local_reader *r);
int hdfs3_local_reader_stats(hdfs3_local_reader *r, uint32_t *bytes_per_checksum, int *checksum_type,
                             uint64_t *gpu_batches);
/* windows whose pages were DMA'd straight from the mmap'd block file (mapped mode: the
 * default when the read starts on a page and buffer_size is a page multiple; environment
 * HDFS3_LOCAL_MMAP=0 disables it). The others were staged by pread into pinned windows. */
uint64_t hdfs3_local_reader_mapped_windows(hdfs3_local_reader *r);
int hdfs3_local_reader_close(hdfs3_local_reader *r);

/* ------------------------------------------------------------------------------------
 * Output stream: the hdfsWrite / hdfsFlush / hdfsSync / hdfsTell / hdfsCloseFile surface
 * (Hdfs.cpp:864-922) over OutputStreamImpl's append/flush/close (OutputStreamImpl.cpp:
 * 298-441, 512-575). Every chunk's CRC32C is computed on the GPU in batches of packets
 * (compute-on-write) and every packet handed to the sink is byte-identical to
 * Packet::getBuffer (Packet.cpp:124-153): [31 B PacketHeader][chunks x BE32 CRC][data],
 * same seqno/offsetInBlock/lastPacketInBlock sequence, the flushed partial chunk re-sent
 * by the next packet, the empty last packet closing every block.
 *
 * The sink is where PipelineImpl::send (Pipeline.cpp:621-678) plugs in: packets arrive
 * in seqno order, batch_packets at a time (and at every flush/sync/close, which return
 * only after the sink received everything written so far). A non-zero sink return fails
 * the stream (sticky, like OutputStreamImpl::setError).
 * Error convention: hdfs.h's (-1 with errno) for write/flush/sync/tell/close.
 * ---------------------------------------------------------------------------------- */
typedef struct hdfs3_output_stream hdfs3_output_stream;

typedef struct hdfs3_packet_info {
    int64_t seqno;
    int64_t offset_in_block;
    int64_t block_index;         /* 0 for the first block of the stream                */
    int32_t data_len;
    int32_t num_chunks;
    int32_t last_packet_in_block;
} hdfs3_packet_info;

/* returns 0, or -errno to fail the stream; `packet` is valid only during the call */
typedef int (*hdfs3_packet_sink)(void *user, const void *packet, size_t len, const hdfs3_packet_info *info);

typedef struct hdfs3_writer_opts {
    int device;
    uint32_t bytes_per_checksum;  /* dfs.bytes-per-checksum (512)                      */
    int32_t packet_size;          /* dfs.client-write-packet-size (65536)               */
    int64_t block_size;           /* dfs.default.blocksize; a multiple of the chunk size */
    int batch_packets;            /* packets per GPU batch (64)                         */
} hdfs3_writer_opts;

/* 0 or -errno; -EINVAL for a packet size below the chunk size or a block size that is
 * not a multiple of it (OutputStreamImpl.cpp:258-273) */
int hdfs3_output_open(const hdfs3_writer_opts *opts, hdfs3_packet_sink sink, void *user,
                      hdfs3_output_stream **out);
/* Append (hdfsOpenFile with O_APPEND; OutputStreamImpl::initAppend, OutputStreamImpl.cpp:172-230):
 * what the namenode's append() returns, supplied by the caller (the namenode is out of scope).
 * The stream's tell() starts at file_length; the appended block's packets start at
 * offsetInBlock = last_block_bytes. A file ending mid-chunk gets a first packet of ONE chunk of
 * chunkSize - file_length % chunkSize bytes with its CRC over those bytes only; a file ending on a
 * chunk boundary gets a first packet capped at the block's free space; the configured sizes return
 * after the first full packet (:332-337). -EIO when the last block is already full (:191-196). */
typedef struct hdfs3_append_info {
    int64_t file_length;       /* FileStatus::getLength                                          */
    int64_t last_block_bytes;  /* the last block's getNumBytes; -1 when append() returned no last
                                  block (the file ends on a block boundary: writes start a new one) */
} hdfs3_append_info;
int hdfs3_output_open_append(const hdfs3_writer_opts *opts, const hdfs3_append_info *append, hdfs3_packet_sink sink,
                             void *user, hdfs3_output_stream **out);
int32_t hdfs3_output_write(hdfs3_output_stream *s, const void *buf, int32_t len);  /* hdfsWrite: len or -1 */
int hdfs3_output_flush(hdfs3_output_stream *s);    /* hdfsFlush / hdfsHFlush: flushInternal(false) */
int hdfs3_output_sync(hdfs3_output_stream *s);     /* hdfsSync: flushInternal(true)               */
int64_t hdfs3_output_tell(hdfs3_output_stream *s);
int hdfs3_output_stats(hdfs3_output_stream *s, uint64_t *packets, uint64_t *gpu_batches);
/* hdfsCloseFile: the remaining packets and the block's last packet reach the sink; frees s */
int hdfs3_output_close(hdfs3_output_stream *s);

/* ------------------------------------------------------------------------------------
 * Write pipeline: PipelineImpl (src/client/Pipeline.cpp) for the blocks of one file, the
 * transport PipelineImpl::send plugs into the sink above. Per block it connects to the
 * first node, sends OP_WRITE_BLOCK (stage PIPELINE_SETUP_CREATE, the remaining nodes as
 * targets, ChecksumProto{CRC32C, bytes_per_checksum}; DataTransferProtocolSender.cpp:
 * 125-150) and checks the BlockOpResponseProto (createBlockOutputStream, Pipeline.cpp:
 * 529-608); then writes each packet and consumes PipelineAckProto acks (one status per
 * node) on the caller's thread: one non-blocking check after every send, blocking when more
 * than max_unacked packets are outstanding, at flush and around the block's last packet
 * (send/checkResponse/waitForAcks/close, :621-841).
 *
 * `blocks` stands in for the namenode: blocks[i] is what addBlock would return for the
 * file's i-th block (its id and the pipeline's nodes, first node first); the byte counts
 * and offsets of hdfs3_located_block are ignored here. Pipeline recovery (a namenode round,
 * :610-619 and buildForAppendOrRecovery) is not rebuilt: any failure — an error status in an
 * ack, a bad connect ack, a seqno out of order, a timeout — is sticky and surfaces as -EIO
 * with the message the reference throws before it starts recovery
 * ("processAck: ack report error at node: ...", "Bad connect ack with firstBadLink as ...").
 * ---------------------------------------------------------------------------------- */
typedef struct hdfs3_pipeline hdfs3_pipeline;

typedef struct hdfs3_pipeline_opts {
    int timeout_ms;      /* output.read.timeout / output.write.timeout analogue (60 s)       */
    int max_unacked;     /* output.packetpool.size (1024, SessionConfig.cpp:126)            */
    int checksum_type;   /* 0 or 2 (CHECKSUM_CRC32C, the only type the output stream makes) */
} hdfs3_pipeline_opts;

int hdfs3_pipeline_open(const hdfs3_located_block *blocks, int n_blocks, const char *client_name,
                        uint32_t bytes_per_checksum, const hdfs3_pipeline_opts *opts, hdfs3_pipeline **out);
/* PipelineImpl(append = true) (Pipeline.cpp:58-81): blocks[0] is the file's last block as append()
 * returned it (id, generation stamp, num_bytes = its length, its replicas as the pipeline nodes);
 * its pipeline is set up with stage PIPELINE_SETUP_APPEND, minBytesRcvd = maxBytesRcvd = num_bytes
 * and latestGenerationStamp = new_generation_stamp (updateBlockForPipeline's, :274-276), after
 * which the block carries that stamp (lastBlock = lb, :327-334). blocks[1..] are the blocks
 * addBlock allocates once it is full (PIPELINE_SETUP_CREATE). */
int hdfs3_pipeline_open_append(const hdfs3_located_block *blocks, int n_blocks, uint64_t new_generation_stamp,
                               const char *client_name, uint32_t bytes_per_checksum,
                               const hdfs3_pipeline_opts *opts, hdfs3_pipeline **out);
/* block i's generation stamp as the pipeline left it (the new stamp for an appended block) */
int hdfs3_pipeline_generation_stamp(hdfs3_pipeline *p, int block, uint64_t *gs);
/* an hdfs3_packet_sink (pass the pipeline as `user`): PipelineImpl::send, or ::close for a
 * block's last packet (waits for every ack of the block, then closes its connection) */
int hdfs3_pipeline_send(void *pipeline, const void *packet, size_t len, const hdfs3_packet_info *info);
/* PipelineImpl::flush: waitForAcks(true) */
int hdfs3_pipeline_flush(hdfs3_pipeline *p);
/* bytes acked per block (lastBlock->setNumBytes(bytesAcked)), packets sent, acks received */
int hdfs3_pipeline_stats(hdfs3_pipeline *p, int64_t *block_bytes_acked, int n_blocks, uint64_t *packets,
                         uint64_t *acks);
/* the sticky failure's message ("" while healthy) */
const char *hdfs3_pipeline_error(hdfs3_pipeline *p);
/* waits for outstanding acks, closes the connection and frees p; 0 or the sticky -errno */
int hdfs3_pipeline_close(hdfs3_pipeline *p);

/* hdfs3_output_open with the pipeline as its sink, plus PipelineImpl::flush at every
 * flush/sync (OutputStreamImpl::flushInternal, :438-440): hdfsFlush/hdfsSync return after
 * every node acked everything written so far. The pipeline's bytes_per_checksum must equal
 * opts->bytes_per_checksum (-EINVAL). The stream does not own the pipeline. */
int hdfs3_output_open_pipeline(const hdfs3_writer_opts *opts, hdfs3_pipeline *pipeline,
                               hdfs3_output_stream **out);
/* the same over a pipeline opened by hdfs3_pipeline_open_append (or hdfs3_pipeline_open when
 * append->last_block_bytes < 0) */
int hdfs3_output_open_pipeline_append(const hdfs3_writer_opts *opts, const hdfs3_append_info *append,
                                      hdfs3_pipeline *pipeline, hdfs3_output_stream **out);

/* ------------------------------------------------------------------------------------
 * OP_BLOCK_CHECKSUM client (DataTransferProtocolSender::blockChecksum, a TODO in the
 * reference, DataTransferProtocolSender.cpp:169-180): sends version | 85 | varint len |
 * OpBlockChecksumProto to host:port and parses BlockOpResponseProto.checksumResponse
 * (datatransfer.proto:189-227). A non-SUCCESS status or a reply without the checksum
 * response fails with -EIO (message in hdfs3_crc_last_error), a malformed reply with
 * -EPROTO. Compare md5 with hdfs3_block_checksum_dev over the same block to check a
 * replica end to end.
 * ---------------------------------------------------------------------------------- */
typedef struct hdfs3_block_checksum_info {
    uint32_t bytes_per_crc;
    uint64_t crc_per_block;
    uint8_t md5[16];
    int crc_type;                 /* ChecksumTypeProto, or -1 when the reply omits it */
} hdfs3_block_checksum_info;

int hdfs3_block_checksum_remote(const char *host, int port, const hdfs3_block_id *block, int timeout_ms,
                                hdfs3_block_checksum_info *out);

#ifdef __cplusplus
}
#endif
#endif /* HDFS3_CLIENT_H */
