/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (bench.py's config-5 CPU baseline leg).
 *
 * The reference's read loop for one block, on one thread, over an OP_READ_BLOCK
 * connection whose request and BlockOpResponseProto the caller already exchanged:
 * RemoteBlockReader::readNextPacket (src/client/RemoteBlockReader.cpp:226-277) reads the
 * fixed-size packet header (PacketHeader::GetPkgHeaderSize(), 31 bytes), then the packet's
 * [checksums][data] into one buffer (:244-245), verifies every chunk with the engine
 * (verifyChecksum, :306-326: a short tail chunk's mismatch is ignored), and read()
 * (:332-357) copies the packet's data to the caller. The empty last packet ends the
 * block (readTrailingEmptyPacket, :279-287). Included by crc32c_oracle.c (the restated
 * engines) and ref_driver.cpp (the reference's own HWCrc32c).
 */
#ifndef HDFS3_ORACLE_REMOTE_LOOP_H
#define HDFS3_ORACLE_REMOTE_LOOP_H

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>

/* first bad chunk of [data, data+len) against the BE words, or -1 (check_short_tail = 0) */
typedef int64_t (*remote_loop_verify_fn)(void *user, const void *data, int64_t len, int bpc, const void *crc_be);

static int remote_loop_recv(int fd, unsigned char *p, size_t n) {
    while (n) {
        ssize_t r = recv(fd, p, n, MSG_WAITALL);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return -1;
        p += r;
        n -= (size_t)r;
    }
    return 0;
}

static uint64_t remote_loop_varint(const unsigned char *b, size_t n, size_t *i) {
    uint64_t v = 0;
    for (int s = 0; *i < n && s < 64; s += 7) {
        unsigned char c = b[(*i)++];
        v |= (uint64_t)(c & 0x7F) << s;
        if (!(c & 0x80)) break;
    }
    return v;
}

/* PacketHeaderProto (datatransfer.proto): offsetInBlock = 1 (sfixed64), seqno = 2 (sfixed64),
 * lastPacketInBlock = 3 (bool), dataLen = 4 (sfixed32), syncBlock = 5 (bool) */
static int remote_loop_header(const unsigned char *h, int32_t *packet_len, int32_t *data_len, int *last) {
    *packet_len = (int32_t)(((uint32_t)h[0] << 24) | ((uint32_t)h[1] << 16) | ((uint32_t)h[2] << 8) | h[3]);
    size_t plen = ((size_t)h[4] << 8) | h[5], i = 0;
    if (plen > 25) return -1;
    const unsigned char *b = h + 6;
    *data_len = -1;
    *last = 0;
    while (i < plen) {
        uint64_t key = remote_loop_varint(b, plen, &i);
        unsigned f = (unsigned)(key >> 3), wt = (unsigned)(key & 7);
        if (wt == 0) {
            uint64_t v = remote_loop_varint(b, plen, &i);
            if (f == 3) *last = v != 0;
        } else if (wt == 1) {
            i += 8;
        } else if (wt == 5) {
            if (i + 4 > plen) return -1;
            int32_t v;
            memcpy(&v, b + i, 4);
            if (f == 4) *data_len = v;
            i += 4;
        } else {
            return -1;
        }
    }
    return *data_len < 0 ? -1 : 0;
}

/* Returns the bytes delivered to `out` (at most cap), -1 on a socket or protocol error.
 * *bad_packet = index of the first packet whose verify failed (the loop stops there, as the
 * reference throws ChecksumException), else -1. verify = 0: transport and copies only. */
static int64_t remote_loop_read_block(int fd, void *out, int64_t cap, int bpc, int verify, int64_t *bad_packet,
                                      remote_loop_verify_fn fn, void *user) {
    unsigned char hdr[31];
    unsigned char *buffer = NULL;
    size_t buf_cap = 0;
    int64_t got = 0, pk = 0;
    *bad_packet = -1;
    for (;; ++pk) {
        int32_t packet_len, data_len;
        int last;
        if (remote_loop_recv(fd, hdr, sizeof hdr) || remote_loop_header(hdr, &packet_len, &data_len, &last)) goto fail;
        if (data_len == 0) break; /* the empty last packet */
        int64_t chunks = ((int64_t)data_len + bpc - 1) / bpc;
        size_t size = (size_t)(chunks * 4 + data_len);
        if ((int64_t)packet_len != 4 + (int64_t)size || got + data_len > cap) goto fail;
        if (size > buf_cap) { /* buffer.resize(size) */
            free(buffer);
            buffer = (unsigned char *)malloc(size);
            if (!buffer) goto fail;
            buf_cap = size;
        }
        if (remote_loop_recv(fd, buffer, size)) goto fail;
        if (verify && fn(user, buffer + chunks * 4, data_len, bpc, buffer) >= 0) {
            *bad_packet = pk;
            break;
        }
        memcpy((unsigned char *)out + got, buffer + chunks * 4, (size_t)data_len);
        got += data_len;
    }
    free(buffer);
    return got;
fail:
    free(buffer);
    return -1;
}

#endif
