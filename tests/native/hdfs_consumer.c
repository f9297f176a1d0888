/* A plain C caller of libhdfs3's hdfs.h surface (include/hdfs3_hdfs.h, prototypes of
 * src/client/hdfs.h:80-436), written the way the reference's function tests use the C API
 * (test/function/TestCInterface.cpp): hdfsOpenFile / hdfsWrite / hdfsFlush / hdfsSync /
 * hdfsCloseFile, then hdfsOpenFile / hdfsRead / hdfsPread / hdfsSeek / hdfsTell /
 * hdfsAvailable, and the errno of each failure path.
 *
 * Write: FillBuffer data ("012345678\n", mock/TestUtil.h:44-53) goes through hdfsWrite; the
 * GPU computes every chunk's CRC32C and the packets arrive at a sink (the write pipeline's
 * place), where their words are checked against the oracle (test infrastructure) and
 * reassembled into blocks. Read: loopback datanodes (tools/loopback, test infrastructure)
 * serve those blocks with the GPU-written words over TCP; the file is read back through
 * hdfsRead with the corrupt replica listed first (one failover), and with only the corrupt
 * replica (-1 / EIO after the good bytes).
 *
 *   hdfs_consumer                      1 MiB blocks, 1 KiB packets, 3 blocks + 234 B
 *   hdfs_consumer BLOCK_MIB N_BLOCKS   e.g. 128 8: BASELINE.json configs[4], the 1 GiB file
 *                                      of 8 x 128 MiB blocks, 64 KiB packets; prints the
 *                                      end-to-end hdfsRead rate
 * exit 0 = every check passed (needs a gfx950 device). */
#define _GNU_SOURCE
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "crc32c_oracle.h"
#include "hdfs3_crc.h"
#include "hdfs3_hdfs.h"

/* tools/loopback/loopback_datanode.cpp (libhdfs3_loopback.so) */
int hdfs3_loopback_start(int *port);
int hdfs3_loopback_add_block(int port, uint64_t block_id, const void *data, uint64_t len, const void *crc_be,
                             uint32_t bpc, int checksum_type);
int hdfs3_loopback_set_packet_bytes(int port, int n);
int hdfs3_loopback_stop(int port);

static int g_fail = 0;
#define CHECK(cond, ...)                                          \
    do {                                                          \
        if (!(cond)) {                                            \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);  \
            fprintf(stderr, __VA_ARGS__);                         \
            fprintf(stderr, "\n");                                \
            ++g_fail;                                             \
        }                                                         \
    } while (0)

static const char kPat[] = "012345678\n";
static void fill_buffer(uint8_t *p, size_t n, size_t offset) {
    for (size_t i = 0; i < n; ++i) p[i] = (uint8_t)kPat[(offset + i) % 10];
}
static int check_buffer(const uint8_t *p, size_t n, size_t offset) {
    for (size_t i = 0; i < n; ++i)
        if (p[i] != (uint8_t)kPat[(offset + i) % 10]) return 0;
    return 1;
}
static uint32_t be32(const uint8_t *p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

#define BPC 512u
#define MAX_BLOCKS 64

/* the write pipeline's place: packets reassembled into blocks + their words */
struct collected {
    int64_t block_size;
    uint8_t *data[MAX_BLOCKS], *crc[MAX_BLOCKS];
    int64_t len[MAX_BLOCKS];
    int64_t packets, last_packets, next_seqno, nblocks;
};

static int sink(void *user, const void *packet, size_t len, const hdfs3_packet_info *info) {
    struct collected *c = (struct collected *)user;
    const uint8_t *p = (const uint8_t *)packet;
    const size_t nch = (size_t)info->num_chunks, dl = (size_t)info->data_len;
    CHECK(len == 31 + 4 * nch + dl, "packet length %zu", len);
    CHECK(be32(p) == dl + 4 * nch + 4, "packetLen field %u", be32(p));  /* Packet.cpp:146-147 */
    CHECK(info->seqno == c->next_seqno, "seqno %lld", (long long)info->seqno);
    c->next_seqno = info->seqno + 1;
    ++c->packets;
    c->last_packets += info->last_packet_in_block ? 1 : 0;
    const int64_t b = info->block_index;
    if (b < 0 || b >= MAX_BLOCKS) {
        CHECK(0, "block index %lld", (long long)b);
        return -EINVAL;
    }
    if (!c->data[b]) {
        c->data[b] = (uint8_t *)malloc((size_t)c->block_size);
        c->crc[b] = (uint8_t *)malloc((size_t)(c->block_size / BPC + 1) * 4);
        if (b + 1 > c->nblocks) c->nblocks = b + 1;
    }
    if (!dl) return 0;  /* the block's empty last packet */
    const uint8_t *words = p + 31, *data = words + 4 * nch;
    uint8_t want[4 * 256];
    if (nch <= 256) {
        oracle_compute_chunks(1, data, dl, BPC, want);
        CHECK(memcmp(words, want, 4 * nch) == 0, "packet %lld: GPU CRC words differ from the oracle",
              (long long)info->seqno);
    }
    /* a flushed partial chunk is re-sent by the next packet from its chunk start */
    CHECK(info->offset_in_block % BPC == 0 && info->offset_in_block <= c->len[b], "offsetInBlock %lld",
          (long long)info->offset_in_block);
    memcpy(c->data[b] + info->offset_in_block, data, dl);
    memcpy(c->crc[b] + info->offset_in_block / BPC * 4, words, 4 * nch);
    c->len[b] = info->offset_in_block + (int64_t)dl;
    return 0;
}

int main(int argc, char **argv) {
    const int64_t block_mib = argc > 1 ? atoll(argv[1]) : 1;
    const int64_t nfull = argc > 2 ? atoll(argv[2]) : 3;
    const int big = argc > 1;
    const int64_t block_size = block_mib << 20;
    const int64_t size = nfull * block_size + (big ? 0 : 234);
    const int32_t packet = big ? 65536 : 1024;
    if (nfull + 1 > MAX_BLOCKS || block_mib <= 0) return 2;

    hdfs3_reader_opts ro = {0, 1, 64, 20000};
    hdfs3_writer_opts wo = {0, BPC, packet, block_size, 64};
    hdfsFS fs = hdfs3_fs_new("hdfs_consumer", &ro, &wo);
    CHECK(fs != NULL, "hdfs3_fs_new");
    if (!fs) return 1;

    /* ---- error paths of hdfsOpenFile (Hdfs.cpp:650-654) ----------------------------- */
    errno = 0;
    CHECK(hdfsOpenFile(fs, "/tmp/f", O_RDWR, 0, 0, 0) == NULL && errno == ENOTSUP, "O_RDWR: errno %d", errno);
    errno = 0;
    CHECK(hdfsOpenFile(fs, "/missing", O_RDONLY, 0, 0, 0) == NULL && errno == ENOENT, "missing: errno %d", errno);
    errno = 0;
    CHECK(hdfsOpenFile(NULL, "/tmp/f", O_RDONLY, 0, 0, 0) == NULL && errno == EINVAL, "null fs: errno %d", errno);
    CHECK(hdfsExists(fs, "/tmp/f") == -1, "exists before write");

    /* ---- write ------------------------------------------------------------------------ */
    struct collected c;
    memset(&c, 0, sizeof(c));
    c.block_size = block_size;
    CHECK(hdfs3_fs_set_sink(fs, "/tmp/f", sink, &c) == 0, "set_sink");
    hdfsFile out = hdfsOpenFile(fs, "/tmp/f", O_WRONLY | O_CREAT, 0, 0, 0);
    CHECK(out != NULL, "open for write: %s", hdfsGetLastError());
    CHECK(out && hdfsFileIsOpenForWrite(out) == 1 && hdfsFileIsOpenForRead(out) == 0, "open mode");
    const size_t wchunk = big ? ((size_t)4 << 20) : 64 * 1024;
    uint8_t *buf = (uint8_t *)malloc(wchunk);
    int64_t off = 0;
    int nw = 0;
    const double tw0 = now_s();
    while (out && off < size) {
        const tSize b = (tSize)(size - off < (int64_t)wchunk ? size - off : (int64_t)wchunk);
        fill_buffer(buf, (size_t)b, (size_t)off);
        CHECK(hdfsWrite(fs, out, buf, b) == b, "hdfsWrite at %lld: %s", (long long)off, hdfsGetLastError());
        off += b;
        if (!big && ++nw % 7 == 0) CHECK(hdfsFlush(fs, out) == 0, "hdfsFlush");  /* partial chunks re-sent */
        if (!big && nw == 10) CHECK(hdfsSync(fs, out) == 0, "hdfsSync");
    }
    errno = 0;
    CHECK(out && hdfsRead(fs, out, buf, 10) == -1 && errno == EINVAL, "hdfsRead on a write file: errno %d", errno);
    CHECK(out && hdfsTell(fs, out) == size, "hdfsTell after write");
    CHECK(out && hdfsCloseFile(fs, out) == 0, "hdfsCloseFile (write)");
    const double tw = now_s() - tw0;
    CHECK(c.nblocks == nfull + (size % block_size ? 1 : 0), "%lld blocks written", (long long)c.nblocks);
    CHECK(c.last_packets == c.nblocks, "%lld last packets", (long long)c.last_packets);
    int64_t total = 0;
    for (int64_t b = 0; b < c.nblocks; ++b) {
        CHECK(check_buffer(c.data[b], (size_t)c.len[b], (size_t)total), "block %lld content", (long long)b);
        total += c.len[b];
    }
    CHECK(total == size, "%lld bytes written", (long long)total);

    /* ---- serve: good replica + a replica with one flipped bit in block 1 -------------- */
    int good = 0, bad = 0;
    CHECK(hdfs3_loopback_start(&good) == 0 && hdfs3_loopback_start(&bad) == 0, "loopback start");
    hdfs3_loopback_set_packet_bytes(good, packet);
    hdfs3_loopback_set_packet_bytes(bad, packet);
    const int64_t flip = c.len[1] / 2 + 17;
    hdfs3_datanode both[2] = {{"127.0.0.1", bad}, {"127.0.0.1", good}};
    hdfs3_datanode only_bad[1] = {{"127.0.0.1", bad}};
    hdfs3_located_block lbs[MAX_BLOCKS], lbs_bad[MAX_BLOCKS];
    /* the loopback datanode references the buffers it serves: the bad replica's block 1 is a copy */
    uint8_t *corrupt = (uint8_t *)malloc((size_t)c.len[1]);
    memcpy(corrupt, c.data[1], (size_t)c.len[1]);
    corrupt[flip] ^= 0x20;
    off = 0;
    for (int64_t b = 0; b < c.nblocks; ++b) {
        const uint64_t id = 7000 + (uint64_t)b;
        hdfs3_loopback_add_block(good, id, c.data[b], (uint64_t)c.len[b], c.crc[b], BPC, 2);
        hdfs3_loopback_add_block(bad, id, b == 1 ? corrupt : c.data[b], (uint64_t)c.len[b], c.crc[b], BPC, 2);
        hdfs3_block_id bid = {"BP-loopback", id, 1, (uint64_t)c.len[b]};
        hdfs3_located_block lb = {bid, off, both, 2};
        lbs[b] = lb;
        lbs_bad[b] = lb;
        lbs_bad[b].replicas = only_bad;
        lbs_bad[b].n_replicas = 1;
        off += c.len[b];
    }
    CHECK(hdfs3_fs_add_file(fs, "/tmp/f", lbs, (int)c.nblocks) == 0, "add_file");
    CHECK(hdfs3_fs_add_file(fs, "/tmp/bad", lbs_bad, (int)c.nblocks) == 0, "add_file bad");
    CHECK(hdfsExists(fs, "/tmp/f") == 0, "exists");

    /* ---- read the whole file: hdfsRead, CheckBuffer, one failover ---------------------- */
    hdfsFile in = hdfsOpenFile(fs, "/tmp/f", O_RDONLY, 0, 0, 0);
    CHECK(in != NULL, "open for read: %s", hdfsGetLastError());
    CHECK(in && hdfsFileIsOpenForRead(in) == 1, "read mode");
    const size_t rchunk = big ? ((size_t)4 << 20) : 20 * 1024 + 1;  /* TestInputStream.cpp:256-273 */
    uint8_t *rbuf = (uint8_t *)malloc(rchunk);
    off = 0;
    const double tr0 = now_s();
    while (in && off < size) {
        const tSize want = (tSize)(size - off < (int64_t)rchunk ? size - off : (int64_t)rchunk);
        const tSize got = hdfsRead(fs, in, rbuf, want);
        CHECK(got > 0, "hdfsRead at %lld returned %d (%s)", (long long)off, got, hdfsGetLastError());
        if (got <= 0) break;
        if (!check_buffer(rbuf, (size_t)got, (size_t)off)) {
            CHECK(0, "CheckBuffer at %lld", (long long)off);
            break;
        }
        off += got;
    }
    const double tr = now_s() - tr0;
    CHECK(off == size, "read %lld of %lld bytes", (long long)off, (long long)size);
    CHECK(in && hdfsRead(fs, in, rbuf, 10) == 0, "hdfsRead at EOF returns 0");
    CHECK(in && hdfsTell(fs, in) == size, "hdfsTell at EOF");
    /* hdfsPread across a block boundary (TestInputStream.cpp CheckFileContentByPread) */
    const tOffset at = c.len[0] - 1000;
    const tSize plen = 300000 < size - at ? 300000 : (tSize)(size - at);
    uint8_t *pbuf = (uint8_t *)malloc((size_t)plen);
    CHECK(in && hdfsPread(fs, in, pbuf, plen, at) == plen && check_buffer(pbuf, (size_t)plen, (size_t)at), "hdfsPread");
    CHECK(in && hdfsSeek(fs, in, 12345) == 0 && hdfsTell(fs, in) == 12345, "hdfsSeek/hdfsTell");
    CHECK(in && hdfsRead(fs, in, rbuf, 100) == 100 && check_buffer(rbuf, 100, 12345), "read after seek");
    CHECK(in && hdfsAvailable(fs, in) >= 0, "hdfsAvailable");
    errno = 0;
    CHECK(in && hdfsSeek(fs, in, size + 1) == -1 && errno == EOVERFLOW, "seek past EOF: errno %d", errno);
    errno = 0;
    CHECK(in && hdfsWrite(fs, in, rbuf, 10) == -1 && errno == EINVAL, "hdfsWrite on a read file: errno %d", errno);
    CHECK(in && hdfsCloseFile(fs, in) == 0, "hdfsCloseFile (read)");

    /* ---- only the corrupt replica: good bytes, then -1 / EIO -------------------------- */
    hdfsFile inb = hdfsOpenFile(fs, "/tmp/bad", O_RDONLY, 0, 0, 0);
    CHECK(inb != NULL, "open bad");
    off = 0;
    tSize got = 0;
    errno = 0;
    while (inb && (got = hdfsRead(fs, inb, rbuf, (tSize)(rchunk < 65536 ? rchunk : 65536))) > 0) {
        if (!check_buffer(rbuf, (size_t)got, (size_t)off)) {
            CHECK(0, "good bytes before the error at %lld", (long long)off);
            break;
        }
        off += got;
    }
    CHECK(got == -1 && errno == EIO, "all replicas bad: read %d errno %d", got, errno);
    CHECK(strlen(hdfsGetLastError()) > 0, "hdfsGetLastError after EIO");
    CHECK(off >= c.len[0] && off <= c.len[0] + flip, "error surfaced at %lld", (long long)off);
    CHECK(inb && hdfsCloseFile(fs, inb) == 0, "close bad");

    /* ---- the same read with block read-ahead (hdfs3_fs_set_readahead): same bytes, same
     * failover off the corrupt replica, read-ahead readers opened for every later block ---- */
    CHECK(hdfs3_fs_set_readahead(fs, 2, 0) == 0, "set_readahead");
    hdfsFile ina = hdfsOpenFile(fs, "/tmp/f", O_RDONLY, 0, 0, 0);
    CHECK(ina != NULL, "open for read-ahead: %s", hdfsGetLastError());
    off = 0;
    const double ta0 = now_s();
    while (ina && off < size) {
        const tSize want = (tSize)(size - off < (int64_t)rchunk ? size - off : (int64_t)rchunk);
        const tSize g = hdfsRead(fs, ina, rbuf, want);
        CHECK(g > 0, "read-ahead hdfsRead at %lld returned %d (%s)", (long long)off, g, hdfsGetLastError());
        if (g <= 0) break;
        if (!check_buffer(rbuf, (size_t)g, (size_t)off)) {
            CHECK(0, "read-ahead CheckBuffer at %lld", (long long)off);
            break;
        }
        off += g;
    }
    const double ta = now_s() - ta0;
    CHECK(off == size, "read-ahead read %lld of %lld bytes", (long long)off, (long long)size);
    CHECK(ina && hdfsRead(fs, ina, rbuf, 10) == 0, "read-ahead EOF");
    CHECK(ina && hdfsCloseFile(fs, ina) == 0, "close read-ahead file");
    CHECK(hdfs3_fs_set_readahead(fs, 0, 0) == 0, "read-ahead off");

    /* through datanodes: hdfsWrite -> GPU CRCs -> OP_WRITE_BLOCK pipeline of 3 loopback
     * nodes (acks per packet, the last node verifies every word) -> hdfsCloseFile registers the
     * file at the acked lengths -> hdfsOpenFile(O_RDONLY) / hdfsRead back from the nodes */
    int dn[3] = {0, 0, 0};
    for (int i = 0; i < 3; ++i) CHECK(hdfs3_loopback_start(&dn[i]) == 0, "loopback start %d", i);
    hdfs3_datanode chain[3] = {{"127.0.0.1", dn[0]}, {"127.0.0.1", dn[1]}, {"127.0.0.1", dn[2]}};
    hdfs3_located_block alloc[MAX_BLOCKS];
    for (int64_t b = 0; b <= nfull; ++b) {
        hdfs3_located_block lb = {{"BP-loopback", (uint64_t)(5000 + b), 1, 0}, 0, chain, 3};
        alloc[b] = lb;
    }
    CHECK(hdfs3_fs_set_pipeline(fs, "/tmp/dn", alloc, (int)nfull + 1) == 0, "set_pipeline");
    hdfsFile wp = hdfsOpenFile(fs, "/tmp/dn", O_WRONLY | O_CREAT, 0, 3, 0);
    CHECK(wp != NULL, "open through datanodes: %s", hdfsGetLastError());
    double tp = now_s();
    for (int64_t off = 0; wp && off < size;) {
        const int32_t b = (int32_t)(size - off < (int64_t)wchunk ? size - off : (int64_t)wchunk);
        fill_buffer(buf, (size_t)b, (size_t)off);
        CHECK(hdfsWrite(fs, wp, buf, b) == b, "pipeline hdfsWrite at %lld: %s", (long long)off, hdfsGetLastError());
        off += b;
        if (!big && (off / (int64_t)wchunk) % 5 == 0) CHECK(hdfsHFlush(fs, wp) == 0, "pipeline hdfsHFlush");
    }
    CHECK(wp && hdfsCloseFile(fs, wp) == 0, "pipeline hdfsCloseFile: %s", hdfsGetLastError());
    tp = now_s() - tp;
    CHECK(hdfsExists(fs, "/tmp/dn") == 0, "written file exists after completeFile");
    hdfsFile rp = hdfsOpenFile(fs, "/tmp/dn", O_RDONLY, 0, 0, 0);
    CHECK(rp != NULL, "open the written file: %s", hdfsGetLastError());
    int64_t roff = 0;
    while (rp && roff < size) {
        const int32_t want = (int32_t)(size - roff < (int64_t)rchunk ? size - roff : (int64_t)rchunk);
        const int32_t got = hdfsRead(fs, rp, rbuf, want);
        if (got <= 0) {
            CHECK(0, "read back at %lld: %d (%s)", (long long)roff, got, hdfsGetLastError());
            break;
        }
        if (!check_buffer(rbuf, (size_t)got, (size_t)roff)) {
            CHECK(0, "read-back content at %lld", (long long)roff);
            break;
        }
        roff += got;
    }
    CHECK(roff == size, "read back %lld of %lld bytes", (long long)roff, (long long)size);
    CHECK(rp && hdfsRead(fs, rp, rbuf, 10) == 0, "read-back EOF");
    CHECK(rp && hdfsCloseFile(fs, rp) == 0, "close read-back");
    for (int i = 0; i < 3; ++i) hdfs3_loopback_stop(dn[i]);

    hdfs3_loopback_stop(good);
    hdfs3_loopback_stop(bad);
    CHECK(hdfsDisconnect(fs) == 0, "hdfsDisconnect");
    for (int64_t b = 0; b < c.nblocks; ++b) {
        free(c.data[b]);
        free(c.crc[b]);
    }
    free(corrupt);
    free(buf);
    free(rbuf);
    free(pbuf);
    if (g_fail) {
        printf("hdfs_consumer FAILED (%d)\n", g_fail);
        return 1;
    }
    printf("{\"hdfs_consumer\": \"ok\", \"bytes\": %lld, \"blocks\": %lld, \"packets\": %lld, "
           "\"hdfsWrite_GiBps\": %.3f, \"hdfsRead_GiBps\": %.3f, \"hdfsRead_readahead2_GiBps\": %.3f, "
           "\"hdfsWrite_3node_pipeline_GiBps\": %.3f}\n",
           (long long)size, (long long)c.nblocks, (long long)c.packets, (double)size / tw / (1 << 30),
           (double)size / tr / (1 << 30), (double)size / ta / (1 << 30), (double)size / tp / (1 << 30));
    return 0;
}
