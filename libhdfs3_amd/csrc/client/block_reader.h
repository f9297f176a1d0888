// Internal entry points of the block reader shared with the input stream.
#pragma once

#include "hdfs3_client.h"
#include "hdfs3_crc.h"

namespace hdfs3crc {

// hdfs3_block_reader_open with an optional borrowed context: the input stream hands its
// own ctx to every block reader it opens (one ctx per stream, SURVEY.md §8b threading).
// slots: depth of the ring of pinned batch arenas the receiver reads ahead into (0 = the
// default 3; the input stream's block read-ahead asks for up to a whole block's worth)
int open_block_reader(const char *host, int port, const hdfs3_block_id *blk, int64_t start, int64_t len,
                      const char *client_name, const hdfs3_reader_opts *opts, hdfs3_crc_ctx *shared_ctx,
                      hdfs3_block_reader **out, int slots = 0, uint8_t *dest = nullptr);

// bytes of one batch arena of a reader with these options (the read-ahead ring depth unit)
int64_t block_reader_batch_bytes(const hdfs3_reader_opts *opts);
// pinned bytes of one batch arena (arena + descriptor staging + result word)
int64_t block_reader_arena_bytes(const hdfs3_reader_opts *opts);

// true when the reader's failure came from this host's GPU or pinned memory (a HIP error),
// not from the datanode: InputStreamImpl's replica failover must not run on it
bool block_reader_local_fault(const hdfs3_block_reader *r);

}  // namespace hdfs3crc
