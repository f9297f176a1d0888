/*
 * hdfs3_crc.h — C-ABI of the MI355X-native per-chunk CRC32C engine for libhdfs3.
 *
 * This is the drop-in boundary for libhdfs3's checksum hot path. The reference
 * has no plugin registry: the engine is picked by #ifdef behind the streaming
 * `Checksum` ABC (src/common/Checksum.h:43-67) at three call sites, each of which
 * runs a per-chunk reset/update/getValue loop on the CPU:
 *
 *   read/remote : RemoteBlockReader::verifyChecksum   src/client/RemoteBlockReader.cpp:306-326
 *   read/local  : LocalBlockReader::readAndVerify     src/client/LocalBlockReader.cpp:138-163
 *   write       : OutputStreamImpl::appendInternal +  src/client/OutputStreamImpl.cpp:298-359
 *                 Packet::addChecksum                 src/client/Packet.cpp:73-81
 *
 * Every entry point below replaces one of those loops with a batched call on a
 * gfx950 kernel. Conventions follow the reference C API
 * (src/client/hdfs.h, src/client/Hdfs.cpp:75-80,826-881): plain pointers and
 * sizes, return 0 on success and a negative errno-style code on failure, never
 * throw across the boundary; the thread-local message is hdfs3_crc_last_error()
 * (cf. hdfsGetLastError, hdfs.h:80).
 *
 * Checksum words are CRC32C (reflected poly 0x82F63B78, init/xorout 0xFFFFFFFF)
 * stored BIG-ENDIAN, one per bytesPerChecksum chunk (src/common/BigEndian.h:43-59).
 * bpc is any positive byte count, as readers accept any bytesPerChecksum > 0 from a
 * datanode (RemoteBlockReader.cpp:150-156) or a .meta header (LocalBlockReader.cpp:110-115);
 * the reference requires a multiple of 512 only for writes (SessionConfig.cpp:112).
 * bpc in {512, 1024, 2048, 4096} on 16-byte aligned data takes the coalesced round kernels, and
 * so do larger multiples of 4096 on the contiguous-block calls (the 4096-byte pieces' CRCs, then a
 * combine kernel); every other size is verified byte-exactly by the chunk-per-lane kernel.
 *
 * Threading: one ctx per stream/thread, like one Checksum instance per reader or
 * writer in the reference. Distinct contexts share nothing but the device.
 */
#ifndef HDFS3_CRC_H
#define HDFS3_CRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDFS3_CRC_ABI_VERSION 1

/* ChecksumTypeProto (hdfs.proto; Checksum.h:34-35). CRC32C is the default of every
 * ctx; CRC32 (zlib polynomial, boost::crc_32_type in the reference, Crc32.h:41-75) is
 * selected per ctx with hdfs3_crc_ctx_set_checksum_type. */
#define HDFS3_CHECKSUM_TYPE_CRC32 1
#define HDFS3_CHECKSUM_TYPE_CRC32C 2

typedef struct hdfs3_crc_ctx hdfs3_crc_ctx;

/* One HDFS data-transfer packet inside a contiguous arena: the wire layout read by
 * RemoteBlockReader::readNextPacket (RemoteBlockReader.cpp:240-245) is
 * [ceil(dataLen/bpc) x BE32 CRC][dataLen bytes]; crc_off/data_off locate both. */
typedef struct hdfs3_pkt_desc {
    uint64_t data_off; /* byte offset of the packet's data region in the arena   */
    uint64_t crc_off;  /* byte offset of the packet's BE32 CRC region            */
    uint32_t data_len; /* PacketHeaderProto.dataLen (datatransfer.proto:143-150)  */
    uint32_t reserved; /* must be 0                                               */
} hdfs3_pkt_desc;

int hdfs3_crc_abi_version(void);
const char *hdfs3_crc_last_error(void);

/* ---- context --------------------------------------------------------------
 * Owns the HIP stream (unless one is attached), the 4 KiB slice-table image in
 * HBM, result slots and the pinned/device staging rings of the host-buffer API.
 * Replaces the per-reader `shared_ptr<Checksum>` construction at
 * RemoteBlockReader.cpp:169-184, LocalBlockReader.cpp:86-98, OutputStreamImpl.cpp:55-66. */
int hdfs3_crc_ctx_create(int device, hdfs3_crc_ctx **out);
void hdfs3_crc_ctx_destroy(hdfs3_crc_ctx *ctx);
/* Pooled create/destroy for callers that make a context per reader or per file, as libhdfs3
 * does (one Checksum per RemoteBlockReader/LocalBlockReader/OutputStreamImpl). create costs
 * milliseconds (stream, table upload, device query); acquire returns a pooled context of
 * `device` (own stream, CRC32C) when one is free, else creates one. release synchronizes the
 * context's stream and returns it to the process-wide pool (thread-safe), or destroys it when
 * the pool is full or the stream reports an error. Never release a context twice, and never
 * mix release with destroy for the same context. */
int hdfs3_crc_ctx_acquire(int device, hdfs3_crc_ctx **out);
void hdfs3_crc_ctx_release(hdfs3_crc_ctx *ctx);
/* The pool's retained pinned host memory is capped process-wide: a released context first gives
 * back cached arenas and staging until the pooled total fits, and is destroyed when it still does
 * not. The cap is HDFS3_POOL_PINNED_MAX (bytes, or with a K/M/G suffix; read once) and defaults to
 * 1 GiB (a read-ahead stream of depth 3 over 128 MiB blocks keeps its rings); 0 pools nothing. The reference holds one packet buffer per reader
 * (RemoteBlockReader.cpp:244) and nothing once it is closed. */
typedef struct hdfs3_crc_pool_stats {
    uint64_t pooled_contexts;   /* idle contexts in the pool                                  */
    uint64_t pinned_bytes;      /* pinned host memory they retain (staging, arenas, results)   */
    uint64_t device_bytes;      /* device memory they retain (tables, staging, arenas)         */
    uint64_t pinned_cap_bytes;  /* the cap above                                               */
} hdfs3_crc_pool_stats;
int hdfs3_crc_pool_stats_get(hdfs3_crc_pool_stats *out);
/* Destroy every pooled (idle) context, returning its pinned and device memory; contexts in use
 * are not affected. Returns the number destroyed. */
int hdfs3_crc_pool_trim(void);

/* NUMA-local placement (docs/DESIGN_HISTORY.md §6), opt-in with HDFS3_NUMA=1: every thread the library runs for
 * a device (the multi-device workers, the block readers' receivers, the local readers' loaders)
 * binds itself to the CPUs of that device's NUMA node, intersected with the process's allowed CPUs,
 * and allocates its pinned staging there. Off by default: on a one-GPU box it slowed loopback reads
 * whose datanode and caller threads were not bound. hdfs3_device_numa_node: the node of `device` from
 * its PCI function (-1 when the platform does not say). hdfs3_numa_cpus: the policy's input for a
 * PCI function under a sysfs tree (sysfs_root "/sys" on a real host): the CPUs of its node, up to
 * max_cpus of them in cpus[]; returns their count, 0 when the node is unknown, or -errno. */
int hdfs3_device_numa_node(int device, int *node);
int hdfs3_numa_cpus(const char *sysfs_root, const char *pci_bdf, int *cpus, int max_cpus);
/* Attach an external hipStream_t (e.g. a framework's current stream); NULL
 * restores the ctx-owned stream. */
int hdfs3_crc_ctx_set_stream(hdfs3_crc_ctx *ctx, void *hip_stream);
void *hdfs3_crc_ctx_get_stream(hdfs3_crc_ctx *ctx);
int hdfs3_crc_ctx_synchronize(hdfs3_crc_ctx *ctx);
/* Polynomial used by every later compute/verify call on this ctx (the hdfs3_crc32c_*
 * names are kept for the default): HDFS3_CHECKSUM_TYPE_CRC32C or _CRC32; -EINVAL else.
 * The same kernels run either way; only the table image differs. */
int hdfs3_crc_ctx_set_checksum_type(hdfs3_crc_ctx *ctx, int type);
int hdfs3_crc_ctx_get_checksum_type(hdfs3_crc_ctx *ctx);
/* Number of checksum kernels this ctx has launched (lets callers/tests prove the
 * GPU path ran). */
uint64_t hdfs3_crc_ctx_kernel_launches(hdfs3_crc_ctx *ctx);

/* ---- host-buffer API (H2D + kernel + D2H through the ctx's pinned ring) ------
 * compute: Packet::addChecksum per chunk (Packet.cpp:73-81) for ceil(len/bpc)
 * chunks, last one possibly short (OutputStreamImpl.cpp:410-419 flush path).
 * verify: *first_bad_chunk = index of the first mismatching chunk or -1.
 *   check_short_tail = 0: RemoteBlockReader semantics (a short tail chunk's
 *   mismatch is ignored, RemoteBlockReader.cpp:319); 1: LocalBlockReader
 *   semantics (tail checked, LocalBlockReader.cpp:149-161).
 * A mismatch is NOT an error (return 0); callers raise ChecksumException
 * (src/common/Exception.h:116-125) from *first_bad_chunk >= 0. */
int hdfs3_crc32c_compute(hdfs3_crc_ctx *ctx, const void *data, size_t len, uint32_t bpc,
                         void *crc_be_out);
int hdfs3_crc32c_verify(hdfs3_crc_ctx *ctx, const void *data, size_t len, uint32_t bpc,
                        const void *crc_be, int check_short_tail, int64_t *first_bad_chunk);

/* ---- device-resident API (pointers in HBM) ---------------------------------
 * _dev: launched on the ctx stream; verify_dev waits for and returns the result.
 * _async: nothing waits; the result lands in a caller-owned device u64 that must
 * be ZERO before the launch: it stays 0 when every chunk matches, otherwise it
 * holds ~first_bad_chunk (decode with hdfs3_crc_decode_result). */
int hdfs3_crc32c_compute_dev(hdfs3_crc_ctx *ctx, const void *d_data, size_t len, uint32_t bpc,
                             void *d_crc_be_out);
int hdfs3_crc32c_verify_dev(hdfs3_crc_ctx *ctx, const void *d_data, size_t len, uint32_t bpc,
                            const void *d_crc_be, int check_short_tail,
                            int64_t *first_bad_chunk);
int hdfs3_crc32c_verify_dev_async(hdfs3_crc_ctx *ctx, const void *d_data, size_t len,
                                  uint32_t bpc, const void *d_crc_be, int check_short_tail,
                                  uint64_t *d_result);
int64_t hdfs3_crc_decode_result(uint64_t result_word);

/* Same as hdfs3_crc32c_verify_dev_async, with launch flags.
 * HDFS3_LAUNCH_OVERLAP_PREVIOUS: the kernel may start before the PREVIOUS operation on
 * the ctx stream has completed (its AQL packet is launched without the barrier bit), so
 * back-to-back verifies of resident blocks overlap one launch's tail with the next one's
 * head instead of draining the GPU between them (docs/DESIGN_HISTORY.md §5). The caller guarantees:
 *   - the previous operation enqueued on the stream is itself a verify launch of this
 *     library (either form), and
 *   - this launch's data, CRC words and zeroed result word were ready before that
 *     previous verify was enqueued.
 * Never pass it for the first verify after any other work on the stream (an upload,
 * a memset of the result word, a kernel of the caller's): that one must be barriered.
 * Verifies only read their inputs and atomically fold into their own result word, so
 * overlapping verifies cannot affect each other's results. Without the flag (0) the
 * call is exactly hdfs3_crc32c_verify_dev_async. */
#define HDFS3_LAUNCH_OVERLAP_PREVIOUS 1u
int hdfs3_crc32c_verify_dev_async_ex(hdfs3_crc_ctx *ctx, const void *d_data, size_t len,
                                     uint32_t bpc, const void *d_crc_be, int check_short_tail,
                                     uint64_t *d_result, uint32_t flags);
/* hdfs3_crc32c_compute_dev with launch flags (compute-on-write over resident blocks).
 * HDFS3_LAUNCH_OVERLAP_PREVIOUS, under the same rule: the previous operation enqueued on
 * the stream is a compute or verify launch of this library, this launch's data was ready
 * before that one was enqueued, and neither launch reads what the other writes (each
 * compute writes only its own CRC array). 0 = exactly hdfs3_crc32c_compute_dev. */
int hdfs3_crc32c_compute_dev_async_ex(hdfs3_crc_ctx *ctx, const void *d_data, size_t len, uint32_t bpc,
                                      void *d_crc_be_out, uint32_t flags);

/* ---- batch of independent device-resident blocks -------------------------------
 * n blocks (each its own data, CRC array and length; chunk counts < 2^32) verified or
 * computed in ONE launch of the segmented wave kernel — the batch form of the calls
 * above, for callers holding several resident blocks (a block scanner, a multi-block
 * read). Each block is checked exactly as hdfs3_crc32c_verify_dev would check it alone;
 * the launch amortises the per-launch head and dispatch gap (docs/DESIGN_HISTORY.md §5).
 * Mismatch key = (block << 32) | chunk: the sync form returns the lexicographically
 * first bad (block, chunk) or -1/-1; the async form leaves ~key (0 when clean) in the
 * caller-zeroed *d_result (hdfs3_crc_decode_result returns the key). */
typedef struct hdfs3_dev_block {
    const void *data;  /* device pointer                                        */
    void *crc_be;      /* device: stored BE32 words (verify) / written (compute) */
    uint64_t len;      /* bytes                                                 */
} hdfs3_dev_block;

int hdfs3_crc32c_verify_blocks_dev(hdfs3_crc_ctx *ctx, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc,
                                   int check_short_tail, int64_t *bad_block, int64_t *bad_chunk);
int hdfs3_crc32c_verify_blocks_dev_async(hdfs3_crc_ctx *ctx, const hdfs3_dev_block *blocks, size_t n,
                                         uint32_t bpc, int check_short_tail, uint64_t *d_result);
int hdfs3_crc32c_compute_blocks_dev(hdfs3_crc_ctx *ctx, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc);

/* ---- independent blocks over several GPUs (BASELINE.json configs[3]) ----------
 * An HDFS block is independent of every other block, so a multi-block job shards with no
 * exchange step: block b goes to device devices[b % n_devices], each device
 * has its own context, HIP stream and host worker thread, and nothing crosses devices (no
 * RCCL, no peer access). The reference has no multi-GPU analogue; it verifies blocks one
 * packet at a time on the reading thread.
 * hdfs3_multi_create: one context and worker per entry of devices[] (normally distinct; a
 * device listed twice gets two workers with their own streams); 0 or -errno.
 * Like a ctx, a hdfs3_multi serves one caller at a time. */
typedef struct hdfs3_multi hdfs3_multi;
int hdfs3_multi_create(const int *devices, int n_devices, hdfs3_multi **out);
void hdfs3_multi_destroy(hdfs3_multi *m);
int hdfs3_multi_device_count(hdfs3_multi *m);
/* Device-resident blocks: blocks[b] must live on devices[b % n_devices] (checked: -EINVAL).
 * Every device verifies its blocks back to back on its own stream (after the first, each
 * launch overlaps its predecessor, HDFS3_LAUNCH_OVERLAP_PREVIOUS), all devices at once;
 * returns when every device is done. first_bad[b] = first mismatching chunk of block b, or
 * -1 (each block checked exactly as hdfs3_crc32c_verify_dev would check it alone). */
int hdfs3_crc32c_verify_blocks_multi(hdfs3_multi *m, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc,
                                     int check_short_tail, int64_t *first_bad);
int hdfs3_crc32c_compute_blocks_multi(hdfs3_multi *m, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc);
/* Host-memory blocks (data and stored words in host memory, pinned or pageable): block b is
 * staged to devices[b % n_devices] through that device's context (hdfs3_crc32c_verify), so
 * the H2D copies of different devices run over their own PCIe links at once. */
typedef struct hdfs3_host_block {
    const void *data;
    const void *crc_be;  /* verify: stored BE32 words; compute: written (cast away const) */
    uint64_t len;
} hdfs3_host_block;
int hdfs3_crc32c_verify_host_multi(hdfs3_multi *m, const hdfs3_host_block *blocks, size_t n, uint32_t bpc,
                                   int check_short_tail, int64_t *first_bad);
int hdfs3_crc32c_compute_host_multi(hdfs3_multi *m, const hdfs3_host_block *blocks, size_t n, uint32_t bpc);

/* ---- packet-stream API -----------------------------------------------------
 * n packets of one block in one arena (wire layout of a5/a6 in SURVEY.md §8a).
 * Verifies every chunk of every packet; on mismatch reports the first bad packet
 * (index into pk[]) and the chunk inside it, else both -1. The host variant
 * stages the arena through the ctx ring; _dev takes an arena already in HBM and
 * a host descriptor array. */
int hdfs3_crc32c_verify_packets(hdfs3_crc_ctx *ctx, const void *arena, size_t arena_len,
                                const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc,
                                int check_short_tail, int64_t *bad_packet,
                                int64_t *bad_chunk);
int hdfs3_crc32c_verify_packets_dev(hdfs3_crc_ctx *ctx, const void *d_arena, size_t arena_len,
                                    const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc,
                                    int check_short_tail, int64_t *bad_packet,
                                    int64_t *bad_chunk);
/* compute side of the packet API (write path, OutputStreamImpl + Packet::getBuffer):
 * fills each packet's CRC region in place. */
int hdfs3_crc32c_compute_packets_dev(hdfs3_crc_ctx *ctx, void *d_arena, size_t arena_len,
                                     const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc);
/* Asynchronous forms of the two calls above (readers with packet rings, a block scanner over a
 * resident arena): one pass over pk[] on the host, descriptors staged in a ring slot of the
 * ctx, nothing waits. *d_result (device, caller-zeroed) receives ~((packet << 32) | chunk) of
 * the first bad chunk, 0 when clean (hdfs3_crc_decode_result returns the key). */
int hdfs3_crc32c_verify_packets_dev_async(hdfs3_crc_ctx *ctx, const void *d_arena, size_t arena_len,
                                          const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc, int check_short_tail,
                                          uint64_t *d_result);
int hdfs3_crc32c_compute_packets_dev_async(hdfs3_crc_ctx *ctx, void *d_arena, size_t arena_len,
                                           const hdfs3_pkt_desc *pk, size_t n, uint32_t bpc);

/* A packet stream at one pitch — the layout of a received-packet ring and of the block
 * reader's arenas: packet i's BE32 words at crc_off + i*pitch and its data at
 * data_off + i*pitch, data_len bytes each except the last (last_len <= data_len).
 * ONE launch with O(1) host work and no descriptor array: when data_len is a power-of-two
 * number of 4 KiB rounds (64 KiB packets: 16) at bpc 512..4096 with 16-B aligned data, the
 * wave kernel walks the packets directly (docs/DESIGN_HISTORY.md §4.2); any other stream is expanded into
 * descriptors once and takes the asynchronous descriptor path. Same result key; flags as
 * hdfs3_crc32c_verify_dev_async_ex (HDFS3_LAUNCH_OVERLAP_PREVIOUS under the same contract). */
typedef struct hdfs3_pkt_stream {
    uint64_t crc_off;   /* packet 0's CRC region                        */
    uint64_t data_off;  /* packet 0's data                              */
    uint64_t pitch;     /* bytes from one packet to the next (> 0 if n > 1) */
    uint64_t n;         /* packets                                      */
    uint32_t data_len;  /* data bytes of every packet but the last      */
    uint32_t last_len;  /* data bytes of the last packet                */
} hdfs3_pkt_stream;
int hdfs3_crc32c_verify_packet_stream_dev_async(hdfs3_crc_ctx *ctx, const void *d_arena, size_t arena_len,
                                                const hdfs3_pkt_stream *ps, uint32_t bpc, int check_short_tail,
                                                uint64_t *d_result, uint32_t flags);
int hdfs3_crc32c_compute_packet_stream_dev_async(hdfs3_crc_ctx *ctx, void *d_arena, size_t arena_len,
                                                 const hdfs3_pkt_stream *ps, uint32_t bpc);

/* ---- streaming shim ---------------------------------------------------------
 * Checksum::update on a raw state (seed 0xFFFFFFFF = reset(), ~state = getValue()),
 * for sub-chunk pieces only: the partial chunk a writer carries across append()
 * calls (OutputStreamImpl.cpp:309-314). Host code; never used by the batch API. */
uint32_t hdfs3_crc32c_update_host(uint32_t state, const void *p, size_t len);

/* ---- block checksum ("MD5 of CRC32", OP_BLOCK_CHECKSUM) --------------------
 * DataTransferProtocolSender::blockChecksum (DataTransferProtocolSender.h:112-120) is a
 * TODO in the reference (DataTransferProtocolSender.cpp:169-180). The datanode answers it
 * with OpBlockChecksumResponseProto {bytesPerCrc, crcPerBlock, md5} (datatransfer.proto:
 * 222-227), md5 being the MD5 digest of the block's stored CRC words: ceil(len/bpc)
 * big-endian words, exactly the .meta file after its 7-byte header (LocalBlockReader.cpp:
 * 64-121). hdfs3_block_checksum_dev computes those words on the GPU (the ctx's checksum
 * type, one compute launch per 4 Mi chunks) and digests them on the host (MD5 is a serial
 * chain); crc_per_block may be NULL. _crcs digests words the caller already holds (a
 * .meta file). The file checksum (MD5MD5CRC32FileChecksum) is the MD5 of the blocks'
 * 16-byte digests, concatenated in block order. All return 0 or -errno. */
int hdfs3_block_checksum_dev(hdfs3_crc_ctx *ctx, const void *d_data, size_t len, uint32_t bpc,
                             uint8_t *md5_out /* 16 B */, uint64_t *crc_per_block);
int hdfs3_block_checksum_crcs(const void *crc_be, uint64_t n_crcs, uint8_t *md5_out /* 16 B */);
int hdfs3_file_checksum_md5md5crc(const uint8_t *block_md5s /* n_blocks x 16 B */, size_t n_blocks,
                                  uint8_t *md5_out /* 16 B */);

/* ---- device memory helpers for FFI callers without a HIP binding ---------- */
int hdfs3_dev_malloc(void **d_ptr, size_t bytes);
int hdfs3_dev_free(void *d_ptr);
int hdfs3_host_malloc_pinned(void **h_ptr, size_t bytes);
int hdfs3_host_free_pinned(void *h_ptr);
int hdfs3_memcpy_h2d(hdfs3_crc_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);
int hdfs3_memcpy_d2h(hdfs3_crc_ctx *ctx, void *h_dst, const void *d_src, size_t bytes);
int hdfs3_memset_dev(hdfs3_crc_ctx *ctx, void *d_dst, int value, size_t bytes);
int hdfs3_device_count(int *count);

#ifdef __cplusplus
}
#endif
#endif /* HDFS3_CRC_H */
