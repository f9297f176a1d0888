// hdfs3_input_stream: InputStreamImpl's read/pread/seek over located blocks with replica
// failover (src/client/InputStreamImpl.cpp), every block read through the GPU-verifying
// hdfs3_block_reader. The C entry points keep hdfs.h's -1/errno convention (Hdfs.cpp:826-862).
//
// Block read-ahead (opt-in, hdfs3_input_set_readahead; the reference opens a block's reader
// only when the cursor reaches the block): entering block i opens the readers of blocks
// i+1 .. i+D as well, each on its own pooled GPU context and with a ring deep enough for
// max_bytes of the block, so their receiver threads read and verify ahead while block i is
// consumed. When the cursor reaches block i+1 its reader simply becomes the current one:
// read(), failover and EIO behave exactly as for a reader opened on demand.
#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <new>
#include <string>
#include <vector>

#include "../ctx.h"
#include "block_reader.h"
#include "hdfs3_client.h"
#include "hdfs3_crc.h"

using namespace hdfs3crc;

namespace {

constexpr int64_t kMaxSkip = 128 * 1024;  // InputStreamImpl.cpp:1146
constexpr int kShallowArenas = 6;  // arenas any pooled ctx keeps (hdfs3_crc.cpp kArenaCacheKeep)

struct Node {
    std::string host;
    int port;
    bool operator==(const Node &o) const { return port == o.port && host == o.host; }
};

struct Block {
    std::string pool;
    hdfs3_block_id id;
    int64_t offset, length;
    std::vector<Node> replicas;
};

// a reader opened ahead of the cursor (block read-ahead) and the pooled ctx it verifies on
struct Ahead {
    int block;
    hdfs3_block_reader *reader;
    hdfs3_crc_ctx *ctx;
    Node node;
};

// hdfs.h convention: errno + -1; the message goes where hdfs3_crc_last_error reads it
int posix_fail(int err, const std::string &msg) {
    fail(-err, "%s", msg.c_str());
    errno = err;
    return -1;
}

}  // namespace

struct hdfs3_input_stream {
    std::vector<Block> blocks;
    int64_t file_length = 0;
    hdfs3_reader_opts opts{0, 1, 0, 0};
    std::string client_name;
    hdfs3_crc_ctx *ctx = nullptr;
    int64_t cursor = 0;
    int64_t end_of_cur_block = 0;
    int cur = -1;
    hdfs3_block_reader *reader = nullptr;
    Node cur_node;
    std::vector<Node> failed;  // failedNodes
    uint64_t failovers = 0, opened = 0;
    std::string last_error;
    int ahead_blocks = 0;           // hdfs3_input_set_readahead
    int64_t ahead_bytes = 0;
    std::deque<Ahead> ahead;        // readers of blocks after `cur`, by block
    hdfs3_crc_ctx *reader_ctx = nullptr;  // the current reader's own ctx when it came from `ahead`
    uint64_t ahead_opened = 0;
    uint64_t ahead_faults = 0;      // read-ahead readers dropped on a local fault and re-read on demand

    ~hdfs3_input_stream() {
        drop_ahead(-1);
        drop_reader();
        if (ctx) ctx_release(ctx);
    }

    void drop_reader() {
        if (reader) hdfs3_block_reader_close(reader);
        reader = nullptr;
        if (reader_ctx) ctx_release(reader_ctx);  // after the reader: its arenas go back into it
        reader_ctx = nullptr;
    }

    static void close_ahead(Ahead &a) {
        hdfs3_block_reader_close(a.reader);
        ctx_release(a.ctx);
    }

    // close the read-ahead readers not in (keep_from, keep_from + ahead_blocks]
    void drop_ahead(int keep_from) {
        for (auto it = ahead.begin(); it != ahead.end();) {
            if (keep_from >= 0 && it->block > keep_from && it->block <= keep_from + ahead_blocks) {
                ++it;
                continue;
            }
            close_ahead(*it);
            it = ahead.erase(it);
        }
    }

    // entering block i: its read-ahead reader (if any) becomes the current reader; readers
    // of i+1 .. i+ahead_blocks are opened where missing. A block whose reader cannot be
    // opened ahead is left to the on-demand path, which owns replica choice and failover.
    void schedule_ahead(int i) {
        for (auto it = ahead.begin(); it != ahead.end(); ++it) {
            if (it->block != i) continue;
            reader = it->reader;
            reader_ctx = it->ctx;
            cur_node = it->node;
            ahead.erase(it);
            break;
        }
        drop_ahead(i);
        if (ahead_blocks <= 0) return;
        const int64_t unit = block_reader_batch_bytes(&opts);
        for (int j = i + 1; j <= i + ahead_blocks && j < int(blocks.size()); ++j) {
            auto at = std::find_if(ahead.begin(), ahead.end(), [&](const Ahead &a) { return a.block >= j; });
            if (at != ahead.end() && at->block == j) continue;
            const Block &b = blocks[size_t(j)];
            if (b.length <= 0 || b.replicas.empty()) continue;
            const int64_t want = std::min<int64_t>(b.length, ahead_bytes > 0 ? ahead_bytes : b.length);
            // the stream's rings (ahead_blocks of them plus the current reader's) fit the pool's pinned
            // cap, so the pool can keep them for the stream's next blocks and the next stream: with
            // whole-block rings, read-ahead 7 over a 1 GiB file pinned new rings on every open
            // (2.8-3.1 GiB/s against 12.6-13.2 with an uncapped pool, profiles/r03/reentry/r3e2e_fix_*)
            // counted in the arenas' real pinned size (block_reader_arena_bytes), after the few arenas
            // every shallow pooled ctx keeps (the stream's own on-demand reader's among them)
            const int64_t arena = block_reader_arena_bytes(&opts);
            const int64_t cap = int64_t(pool_pinned_cap_bytes());
            const int64_t fit = std::max<int64_t>(0, cap - int64_t(kShallowArenas) * arena) /
                                int64_t(ahead_blocks + 1) / arena;
            const int slots = int(std::max<int64_t>(3, std::min<int64_t>({(want + unit - 1) / unit + 1, 64, fit})));
            hdfs3_crc_ctx *c = nullptr;
            if (ctx_acquire(opts.device, &c, true)) break;  // no context to spare: read on demand
            hdfs3_block_id id = b.id;
            id.pool_id = b.pool.c_str();
            hdfs3_block_reader *r = nullptr;
            const Node &n = b.replicas.front();  // choseBestNode with a fresh failed list
            if (open_block_reader(n.host.c_str(), n.port, &id, 0, b.length, client_name.c_str(), &opts, c, &r,
                                  slots)) {
                ctx_release(c);
                continue;
            }
            ++ahead_opened;
            ahead.insert(at, Ahead{j, r, c, n});
        }
    }

    int find_block(int64_t pos) const {  // LocatedBlocks::findBlock
        auto it = std::upper_bound(blocks.begin(), blocks.end(), pos,
                                   [](int64_t p, const Block &b) { return p < b.offset; });
        if (it == blocks.begin()) return -1;
        const int i = int(it - blocks.begin()) - 1;
        return pos < blocks[i].offset + blocks[i].length ? i : -1;
    }

    // choseBestNode (InputStreamImpl.cpp:322-335): first replica not yet failed
    const Node *best_node(const Block &b) const {
        for (const Node &n : b.replicas)
            if (std::find(failed.begin(), failed.end(), n) == failed.end()) return &n;
        return nullptr;
    }

    // setupBlockReader (:364-450) for [start, start+len) of block b; -errno
    int setup(const Block &b, int64_t start, int64_t len, hdfs3_block_reader **out, Node *node,
              uint8_t *dest = nullptr) {
        std::string why;
        for (;;) {
            const Node *n = best_node(b);
            if (!n) {
                last_error = "InputStreamImpl: all nodes have been tried and no valid replica can be read for Block: " +
                             std::to_string(b.id.block_id) + (why.empty() ? "" : " (last: " + why + ")");
                return -EIO;
            }
            hdfs3_block_id id = b.id;
            id.pool_id = b.pool.c_str();
            const int rc = open_block_reader(n->host.c_str(), n->port, &id, start, len, client_name.c_str(), &opts,
                                             ctx, out, 0, dest);
            if (rc == 0) {
                *node = *n;
                ++opened;
                return 0;
            }
            if (rc == -ENOTSUP || rc == -ENOMEM || rc == -ENODEV) {  // not a replica problem: another node cannot help
                last_error = hdfs3_crc_last_error();
                return rc;
            }
            why = hdfs3_crc_last_error();
            failed.push_back(*n);
        }
    }

    void seek_to_block(int i) {  // seekToBlock: new block, fresh failed list
        drop_reader();
        cur = i;
        end_of_cur_block = blocks[i].offset + blocks[i].length;
        failed.clear();
        // a read-ahead reader starts at the block's first byte: usable on sequential entry
        if ((ahead_blocks > 0 || !ahead.empty()) && cursor == blocks[i].offset) schedule_ahead(i);
        else if (!ahead.empty()) drop_ahead(i);
    }

    // readOneBlock (:616-712)
    int32_t read_one_block(uint8_t *buf, int32_t size) {
        const Block &b = blocks[cur];
        for (;;) {
            if (!reader) {
                const int64_t off = cursor - b.offset;
                if (int rc = setup(b, off, b.length - off, &reader, &cur_node)) return rc;
            }
            const int32_t todo = int32_t(std::min<int64_t>(size, end_of_cur_block - cursor));
            const int32_t n = hdfs3_block_reader_read(reader, buf, todo);
            if (n > 0) {
                cursor += n;
                return n;
            }
            // a local GPU/memory fault is not the replica's: report it, do not burn the replicas.
            // A read-ahead reader faults on its own pooled ctx and deep ring, which an on-demand
            // reader does not need: that block is read again on demand from the cursor on the
            // stream's ctx, and only a fault there is reported (same bytes and errors as with
            // read-ahead off)
            if (block_reader_local_fault(reader)) {
                last_error = hdfs3_crc_last_error();
                const bool prefetched = reader_ctx != nullptr;
                drop_reader();
                if (prefetched) {
                    ++ahead_faults;
                    continue;
                }
                return n < 0 ? n : -EIO;
            }
            // ChecksumException or I/O failure: this replica is bad, try another (:682-708)
            ++failovers;
            failed.push_back(cur_node);
            drop_reader();
        }
    }

    int32_t read(uint8_t *buf, int32_t size) {
        if (cursor >= file_length) return 0;  // HdfsEndOfStream -> hdfsRead returns 0
        if (cursor >= end_of_cur_block || cur < 0) {
            const int i = find_block(cursor);
            if (i < 0) return -EIO;
            seek_to_block(i);
        }
        return read_one_block(buf, size);
    }

    // fetchBlockByteRange (:955-1061): the whole range from one replica, else the next
    int fetch_range(const Block &b, int64_t start, int64_t len, uint8_t *out) {
        std::vector<Node> saved;
        saved.swap(failed);
        int rc = 0;
        for (;;) {
            hdfs3_block_reader *r = nullptr;
            Node node;
            // the range's one destination goes to the reader, which copies each packet there while it is hot
            // (round 6; 8 concurrent preads: client CPU per GiB 1.28-1.41x -> 0.98-1.16x the reference
            // loop's, rate within the spread, profiles/r06/r6eg_config5_eager_ab.jsonl).
            // HDFS3_READER_EAGER_COPY=0 (measurement knob) leaves the copy to read()
            const char *ev = getenv("HDFS3_READER_EAGER_COPY");
            const bool eager = !(ev && ev[0] == '0');
            if ((rc = setup(b, start, len, &r, &node, eager ? out : nullptr))) break;
            int64_t got = 0;
            int32_t n = 0;
            while (got < len) {
                n = hdfs3_block_reader_read(r, out + got, int32_t(std::min<int64_t>(len - got, 1 << 30)));
                if (n <= 0) break;
                got += n;
            }
            const bool local = block_reader_local_fault(r);
            if (local) last_error = hdfs3_crc_last_error();
            hdfs3_block_reader_close(r);
            if (got == len) break;
            if (local) {  // this host's GPU, not the replica: no failover
                rc = n < 0 ? n : -EIO;
                break;
            }
            ++failovers;
            failed.push_back(node);
        }
        failed.swap(saved);
        return rc;
    }

    int32_t pread(int64_t pos, uint8_t *buf, int32_t size) {
        if (pos < 0 || pos >= file_length) return -EINVAL;
        const int32_t real = int32_t(std::min<int64_t>(size, file_length - pos));
        int64_t done = 0;
        while (done < real) {
            const int i = find_block(pos + done);
            if (i < 0) return -EIO;
            const Block &b = blocks[i];
            const int64_t start = pos + done - b.offset;
            const int64_t n = std::min<int64_t>(real - done, b.length - start);
            if (int rc = fetch_range(b, start, n, buf + done)) return rc;
            done += n;
        }
        return real;
    }

    int seek(int64_t pos) {  // seekInternal (:1133-1170)
        if (pos == cursor) return 0;
        if (pos > file_length) return -EOVERFLOW;
        if (reader && pos > cursor && pos < end_of_cur_block && pos - cursor <= kMaxSkip) {
            uint8_t scratch[16384];
            bool ok = true;
            while (cursor < pos) {
                const int32_t n = hdfs3_block_reader_read(reader, scratch, int32_t(std::min<int64_t>(sizeof(scratch), pos - cursor)));
                if (n <= 0) {
                    ok = false;
                    break;
                }
                cursor += n;
            }
            if (ok) return 0;
        }
        drop_reader();
        end_of_cur_block = 0;
        cursor = pos;
        return 0;
    }
};

extern "C" {

int hdfs3_input_open(const hdfs3_located_block *blocks, int n_blocks, const char *client_name,
                     const hdfs3_reader_opts *opts, hdfs3_input_stream **out) {
    if (!out || n_blocks < 0 || (n_blocks && !blocks)) return fail(-EINVAL, "invalid argument");
    *out = nullptr;
    hdfs3_input_stream *s = new (std::nothrow) hdfs3_input_stream();
    if (!s) return fail(-ENOMEM, "input stream allocation");
    if (opts) s->opts = *opts;
    s->client_name = client_name ? client_name : "libhdfs3_amd";
    int64_t expect = n_blocks ? blocks[0].offset : 0;
    for (int i = 0; i < n_blocks; ++i) {
        const hdfs3_located_block &lb = blocks[i];
        if (lb.offset != expect || int64_t(lb.block.num_bytes) < 0 || lb.n_replicas < 0 ||
            (lb.n_replicas && !lb.replicas)) {
            delete s;
            return fail(-EINVAL, "located block %d is not contiguous with its predecessor or malformed", i);
        }
        Block b;
        b.pool = lb.block.pool_id ? lb.block.pool_id : "";
        b.id = lb.block;
        b.id.pool_id = nullptr;
        b.offset = lb.offset;
        b.length = int64_t(lb.block.num_bytes);
        for (int k = 0; k < lb.n_replicas; ++k) {
            if (!lb.replicas[k].host) {
                delete s;
                return fail(-EINVAL, "replica %d of block %d has no host", k, i);
            }
            b.replicas.push_back(Node{lb.replicas[k].host, lb.replicas[k].port});
        }
        expect += b.length;
        s->blocks.push_back(std::move(b));
    }
    if (n_blocks && blocks[0].offset != 0) {
        delete s;
        return fail(-EINVAL, "the first block must start at file offset 0");
    }
    s->file_length = expect;
    if (int rc = ctx_acquire(s->opts.device, &s->ctx)) {
        delete s;
        return rc;
    }
    *out = s;
    return 0;
}

int32_t hdfs3_input_read(hdfs3_input_stream *s, void *buf, int32_t len) {
    if (!s || !buf || len <= 0) return posix_fail(EINVAL, "hdfsRead: invalid argument");
    s->last_error.clear();
    const int32_t rc = s->read(static_cast<uint8_t *>(buf), len);
    if (rc < 0) return posix_fail(-rc, s->last_error.empty() ? hdfs3_crc_last_error() : s->last_error);
    return rc;
}

int32_t hdfs3_input_pread(hdfs3_input_stream *s, int64_t pos, void *buf, int32_t len) {
    if (!s || !buf || len <= 0 || pos < 0) return posix_fail(EINVAL, "hdfsPread: invalid argument");
    s->last_error.clear();
    const int32_t rc = s->pread(pos, static_cast<uint8_t *>(buf), len);
    if (rc == -EINVAL) return posix_fail(EINVAL, "hdfsPread: position outside the file");
    if (rc < 0) return posix_fail(-rc, s->last_error.empty() ? hdfs3_crc_last_error() : s->last_error);
    return rc;
}

int hdfs3_input_seek(hdfs3_input_stream *s, int64_t pos) {
    if (!s || pos < 0) return posix_fail(EINVAL, "hdfsSeek: invalid argument");
    if (int rc = s->seek(pos))
        return posix_fail(-rc, "InputStreamImpl: seek over EOF, seek target: " + std::to_string(pos));
    return 0;
}

int64_t hdfs3_input_tell(hdfs3_input_stream *s) {
    if (!s) return posix_fail(EINVAL, "hdfsTell: invalid argument");
    return s->cursor;
}

int hdfs3_input_available(hdfs3_input_stream *s) {
    if (!s) return posix_fail(EINVAL, "hdfsAvailable: invalid argument");
    const int64_t a = s->reader ? hdfs3_block_reader_available(s->reader) : 0;
    return int(std::min<int64_t>(a, 0x7FFFFFFF));
}

int64_t hdfs3_input_length(hdfs3_input_stream *s) { return s ? s->file_length : -1; }

int hdfs3_input_stats(hdfs3_input_stream *s, uint64_t *failovers, uint64_t *readers_opened) {
    if (!s) return fail(-EINVAL, "null stream");
    if (failovers) *failovers = s->failovers;
    if (readers_opened) *readers_opened = s->opened;
    return 0;
}

int hdfs3_input_set_readahead(hdfs3_input_stream *s, int blocks, int64_t max_bytes_per_block) {
    if (!s || blocks < 0 || max_bytes_per_block < 0) return fail(-EINVAL, "invalid argument");
    // every block opened ahead holds a pooled ctx, a connection and a pinned ring at once
    if (blocks > HDFS3_READAHEAD_MAX_BLOCKS)
        return fail(-EINVAL, "read-ahead of %d blocks: at most %d", blocks, HDFS3_READAHEAD_MAX_BLOCKS);
    s->ahead_blocks = blocks;
    s->ahead_bytes = max_bytes_per_block;
    if (blocks == 0) s->drop_ahead(-1);
    return 0;
}

int hdfs3_input_readahead_stats(hdfs3_input_stream *s, uint64_t *prefetch_readers_opened,
                                uint64_t *prefetch_local_faults) {
    if (!s) return fail(-EINVAL, "null stream");
    if (prefetch_readers_opened) *prefetch_readers_opened = s->ahead_opened;
    if (prefetch_local_faults) *prefetch_local_faults = s->ahead_faults;
    return 0;
}

int hdfs3_input_close(hdfs3_input_stream *s) {
    delete s;
    return 0;
}

}  // extern "C"
