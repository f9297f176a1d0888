/*
 * hdfs3_hdfs.h — libhdfs3's C file-I/O surface (src/client/hdfs.h) over the GPU-verified
 * streams of hdfs3_client.h.
 *
 * The file-I/O functions below (hdfsOpenFile ... hdfsAvailable) have exactly the prototypes
 * of the reference's hdfs.h (cited per line), with the same argument checks, return values and
 * errno convention as src/client/Hdfs.cpp: code that reads and writes through an hdfsFS/hdfsFile
 * compiles and links against libhdfs3_crc.so unchanged. tests/test_reference_headers.py compiles
 * the implementation (csrc/client/hdfs_shim.cpp) with the reference's own hdfs.h force-included,
 * so the compiler checks that every definition matches the reference's declaration.
 *
 * NOT provided: hdfsConnect / hdfsConnectAsUser / hdfsBuilderConnect and the rest of the
 * namespace API (hdfsDelete, hdfsRename, hdfsListDirectory, hdfsGetPathInfo, ...). They are
 * ClientProtocol RPC to the namenode, outside the checksum path. A caller obtains its hdfsFS
 * from hdfs3_fs_new instead of hdfsConnect, and registers per path what the namenode would
 * answer:
 *   - getBlockLocations (for O_RDONLY, and append()'s file length and last block):
 *     hdfs3_fs_add_file — read through hdfs3_input_* (datanode OP_READ_BLOCK, GPU verify,
 *     replica failover);
 *   - create/addBlock (for O_WRONLY): hdfs3_fs_set_pipeline (datanodes, OP_WRITE_BLOCK) or
 *     hdfs3_fs_set_sink (a packet sink), fed by hdfs3_output_* with packets byte-identical to
 *     Packet::getBuffer whose CRCs the GPU computed;
 *   - updateBlockForPipeline's new generation stamp (for O_APPEND): hdfs3_fs_set_append_stamp.
 * Those two lines of setup (hdfs3_fs_new + the registrations) replace hdfsConnect; everything
 * after hdfsOpenFile runs as written against hdfs.h.
 */
#ifndef HDFS3_HDFS_H
#define HDFS3_HDFS_H

#include <fcntl.h>
#include <stdint.h>
#include <time.h>

#include "hdfs3_client.h"

#ifdef __cplusplus
extern "C" {
#endif

/* hdfs.h:56-69 */
typedef int32_t tSize;
typedef time_t tTime;
typedef int64_t tOffset;
typedef uint16_t tPort;
struct HdfsFileSystemInternalWrapper;
typedef struct HdfsFileSystemInternalWrapper *hdfsFS;
struct HdfsFileInternalWrapper;
typedef struct HdfsFileInternalWrapper *hdfsFile;

/* ---- the hdfs.h functions (reference prototypes, Hdfs.cpp semantics) ---------------- */
const char *hdfsGetLastError();                                         /* hdfs.h:80  */
int hdfsFileIsOpenForRead(hdfsFile file);                               /* hdfs.h:88  */
int hdfsFileIsOpenForWrite(hdfsFile file);                              /* hdfs.h:96  */
int hdfsDisconnect(hdfsFS fs);                                          /* hdfs.h:303 */
/* O_RDONLY: the registered LocatedBlocks (ENOENT if none); O_WRONLY [| O_CREAT | O_SYNC]:
 * the registered pipeline or sink (ENOENT if none), blocksize 0 = the fs's writer default, which
 * must be a multiple of the chunk size (EINVAL); O_RDWR, O_EXCL|O_CREAT: ENOTSUP (Hdfs.cpp:653);
 * O_WRONLY|O_APPEND: append to the registered file (ENOENT if none): OutputStreamImpl::initAppend
 * (OutputStreamImpl.cpp:172-230) with the file's length and, when it ends inside a block, its last
 * block (file_length % blocksize != 0, blocksize as for O_WRONLY): written through a
 * PIPELINE_SETUP_APPEND pipeline to that block's replicas (or the registered sink), further blocks
 * through hdfs3_fs_set_pipeline's; a clean close registers the whole file for reading again. */
hdfsFile hdfsOpenFile(hdfsFS fs, const char *path, int flags, int bufferSize, short replication,
                      tOffset blocksize);                                /* hdfs.h:319 */
int hdfsCloseFile(hdfsFS fs, hdfsFile file);                            /* hdfs.h:332 */
int hdfsExists(hdfsFS fs, const char *path);                            /* hdfs.h:340 */
int hdfsSeek(hdfsFS fs, hdfsFile file, tOffset desiredPos);             /* hdfs.h:350 */
tOffset hdfsTell(hdfsFS fs, hdfsFile file);                             /* hdfs.h:358 */
tSize hdfsRead(hdfsFS fs, hdfsFile file, void *buffer, tSize length);   /* hdfs.h:374 */
tSize hdfsPread(hdfsFS fs, hdfsFile file, void *buffer, tSize length, tOffset position); /* :391 */
tSize hdfsWrite(hdfsFS fs, hdfsFile file, const void *buffer, tSize length); /* hdfs.h:401 */
int hdfsFlush(hdfsFS fs, hdfsFile file);                                /* hdfs.h:409 */
int hdfsHFlush(hdfsFS fs, hdfsFile file);                               /* hdfs.h:418 */
int hdfsSync(hdfsFS fs, hdfsFile file);                                 /* hdfs.h:427 */
int hdfsAvailable(hdfsFS fs, hdfsFile file);                            /* hdfs.h:436 */

/* ---- the namenode/pipeline stand-in (not in hdfs.h) ---------------------------------
 * hdfs3_fs_new: an empty path table; read_opts/write_opts are the session's defaults
 * (NULL: device 0, verify on, batch 64 / bpc 512, packet 64 KiB, block 128 MiB, batch 64);
 * client_name is the DFSClient name sent in OP_READ_BLOCK. NULL with errno on failure.
 * Release with hdfsDisconnect. */
hdfsFS hdfs3_fs_new(const char *client_name, const hdfs3_reader_opts *read_opts,
                    const hdfs3_writer_opts *write_opts);
/* what getBlockLocations returns for `path` (blocks in file order, contiguous; copied).
 * 0, or -1 with errno (EINVAL). Replaces an existing entry. */
int hdfs3_fs_add_file(hdfsFS fs, const char *path, const hdfs3_located_block *blocks, int n_blocks);
/* where the write pipeline of `path` starts: every packet of a file opened O_WRONLY goes to
 * sink(user, ...) (hdfs3_client.h), in seqno order. 0, or -1 with errno (EINVAL). */
int hdfs3_fs_set_sink(hdfsFS fs, const char *path, hdfs3_packet_sink sink, void *user);
/* write `path` through datanodes instead: blocks[i] is what addBlock would return for the
 * file's i-th block (id + pipeline nodes; sizes and offsets ignored). A file opened O_WRONLY
 * then writes through hdfs3_pipeline (OP_WRITE_BLOCK, acks; include/hdfs3_client.h), and
 * hdfsFlush/hdfsSync return once every node acked. A clean hdfsCloseFile registers the file for
 * reading at the acked block lengths from the same nodes (completeFile + getBlockLocations), so
 * hdfsOpenFile(O_RDONLY)/hdfsRead read back what was written. Takes precedence over a sink.
 * 0, or -1 with errno (EINVAL). */
int hdfs3_fs_set_pipeline(hdfsFS fs, const char *path, const hdfs3_located_block *blocks, int n_blocks);
/* the file's block size as FileStatus::getBlockSize reports it (what O_APPEND continues with,
 * OutputStreamImpl.cpp:196-230); a clean close of a write through hdfs3_fs_set_pipeline records the
 * size it wrote with. Unset for a file of one block: the caller's or the session's size is used.
 * 0, or -1 with errno (EINVAL). */
int hdfs3_fs_set_block_size(hdfsFS fs, const char *path, int64_t block_size);
/* the generation stamp updateBlockForPipeline would give `path`'s last block when it is next
 * opened O_APPEND (Pipeline.cpp:274-276); unset: that block's stamp + 1. 0, or -1 with errno. */
int hdfs3_fs_set_append_stamp(hdfsFS fs, const char *path, uint64_t new_generation_stamp);
/* block read-ahead for files opened for reading from now on (hdfs3_input_set_readahead in
 * hdfs3_client.h; 0 blocks = off, the reference's one-block-at-a-time reading; at most
 * HDFS3_READAHEAD_MAX_BLOCKS). 0, or -1 with errno (EINVAL). */
int hdfs3_fs_set_readahead(hdfsFS fs, int blocks, int64_t max_bytes_per_block);

#ifdef __cplusplus
}
#endif
#endif /* HDFS3_HDFS_H */
