/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of libhdfs3's per-chunk CRC32C path, used exclusively as the
 * checker in tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * Nothing in libhdfs3_amd/ (the product) links, loads or calls this library.
 *
 * Parity pinning: the restatement is checked against
 *   (1) the reference's own known-answer fixtures test/data/checksum{1,2}.in
 *       (copied verbatim as data into tests/golden/), exercised the way
 *       test/unit/TestChecksum.cpp:83-140 does (8 alignments + streamed total);
 *   (2) oracle/_ref/libref_hwcrc32c.so — the reference's HWCrc32c compiled from
 *       /root/reference/src/common/HWCrc32c.cpp by oracle/Makefile (container
 *       only), via tests/golden/make_golden.py's committed fixtures.
 *
 * All references are /root/reference-relative file:line.
 */
#ifndef HDFS3_CRC_ORACLE_H
#define HDFS3_CRC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Raw-state streaming update, Checksum::update semantics (src/common/Checksum.h:43-67):
 * caller seeds with 0xFFFFFFFF (reset) and finalises with ~state (getValue). */

/* Byte-at-a-time table engine: src/common/SWCrc32c.cpp:97-104 (table :47-91). */
uint32_t oracle_crc32c_sw_update(uint32_t state, const void *p, size_t len);
/* SSE4.2 crc32 engine: src/common/HWCrc32c.cpp:116-186 (head align, crc32q loop, tail). */
uint32_t oracle_crc32c_hw_update(uint32_t state, const void *p, size_t len);
/* 3-way interleaved crc32q + PCLMUL combine, behaviour of crc_pcl:
 * src/common/crc_iscsi_v_pcl.asm:93-340, wrapper src/common/IntelAsmCrc32c.cpp:39-42. */
uint32_t oracle_crc32c_pcl_update(uint32_t state, const void *p, size_t len);

/* reset + update + getValue, i.e. one finished CRC32C word. engine: 0=sw 1=hw 2=pcl */
uint32_t oracle_crc32c(int engine, const void *p, size_t len);

/* Batch compute of per-chunk CRCs, big-endian words (Packet::addChecksum,
 * src/client/Packet.cpp:73-81; OutputStreamImpl.cpp:298-359).
 * Writes ceil(len/bpc) words; last chunk may be short. */
void oracle_compute_chunks(int engine, const void *data, size_t len, uint32_t bpc,
                           void *crc_be_out);

/* Batch verify. check_short_tail=0 restates RemoteBlockReader::verifyChecksum
 * (src/client/RemoteBlockReader.cpp:306-326: a mismatch on a short tail chunk is
 * ignored); check_short_tail=1 restates LocalBlockReader::readAndVerify
 * (src/client/LocalBlockReader.cpp:138-163: every chunk, tail included).
 * Returns the index of the first bad chunk, or -1. */
int64_t oracle_verify_chunks(int engine, const void *data, size_t len, uint32_t bpc,
                             const void *crc_be, int check_short_tail);

/* Multi-threaded CPU verify throughput for the bench's cpu_baseline leg: verifies
 * `len` bytes `reps` times split over `threads` threads. Returns seconds elapsed;
 * *bad_out gets the first-bad index seen (-1). */
double oracle_bench_verify(int engine, const void *data, size_t len, uint32_t bpc,
                           const void *crc_be, int threads, int reps, int64_t *bad_out);

/* Deterministic test-data generator shared with tests/util.py (splitmix64). */
void oracle_fill_splitmix(void *dst, size_t len, uint64_t seed);

/* CHECKSUM_CRC32 — Crc32 (src/common/Crc32.h:41-75) wraps boost::crc_32_type, a
 * third-party dependency absent from /root/reference (version unpinned; README: "tested
 * on 1.53+"). Its published parameters: width 32, poly 0x04C11DB7 (reflected
 * 0xEDB88320), init 0xFFFFFFFF, reflect in/out, final xor 0xFFFFFFFF — the zlib CRC-32.
 * Parity unpinned by reference tests (none cover type 1); pinned instead by the standard
 * check value crc32("123456789") = 0xCBF43926 and Python's zlib.crc32 in tests/.
 * Raw-state update with the same reset/getValue convention as the CRC32C engines. */
uint32_t oracle_crc32_update(uint32_t state, const void *p, size_t len);
void oracle_compute_chunks_crc32(const void *data, size_t len, uint32_t bpc, void *crc_be_out);

/* One block of an OP_READ_BLOCK connection (request and response already exchanged) through
 * RemoteBlockReader's receive -> verifyChecksum -> copy loop on the calling thread
 * (src/client/RemoteBlockReader.cpp:226-357; oracle/remote_loop.h), with a restated engine.
 * Returns bytes copied to out, -1 on error; *bad_packet = first packet that failed verify. */
int64_t oracle_remote_read_block(int fd, int engine, void *out, int64_t cap, int bpc, int verify,
                                 int64_t *bad_packet);

#ifdef __cplusplus
}
#endif
#endif
