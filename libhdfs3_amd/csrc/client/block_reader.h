// Internal entry points of the block reader shared with the input stream.
#pragma once

#include "hdfs3_client.h"
#include "hdfs3_crc.h"

namespace hdfs3crc {

// hdfs3_block_reader_open with an optional borrowed context: the input stream hands its
// own ctx to every block reader it opens (one ctx per stream, SURVEY.md §8b threading)
int open_block_reader(const char *host, int port, const hdfs3_block_id *blk, int64_t start, int64_t len,
                      const char *client_name, const hdfs3_reader_opts *opts, hdfs3_crc_ctx *shared_ctx,
                      hdfs3_block_reader **out);

// true when the reader's failure came from this host's GPU or pinned memory (a HIP error),
// not from the datanode: InputStreamImpl's replica failover must not run on it
bool block_reader_local_fault(const hdfs3_block_reader *r);

}  // namespace hdfs3crc
