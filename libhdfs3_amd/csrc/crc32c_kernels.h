// Internal launch interface of the gfx950 CRC32C kernels (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#include <atomic>

namespace hdfs3crc {

// Workgroup geometry: the bank-replicated slice-table image takes 128 KiB of
// the CU's 160 KiB LDS, so one workgroup owns a CU; 1024 threads = 16 waves
// (4 per SIMD) keep the CU's memory pipe and LDS busy.
constexpr int kBlockThreads = 1024;

// The 4 KiB units of a packet stream (PitchWalk, crc32c_wave.h). A packet of whole chunks is
// ceil(bytes / 4096) units; its last unit may be PARTIAL (the writer's 127-chunk packets at bpc
// 512: 65,024 B = 15 whole rounds + 3,584 B, OutputStreamImpl.cpp:161-170): its loads are bounded by
// a buffer resource of ptail bytes, so the lanes past the last whole chunk read zeros and their
// results are dropped. Unit u -> packet u / upp by a multiply-shift (u < 2^31: q = (u * magic) >>
// shift, Granlund-Montgomery with N = 31), so upp need not be a power of two.
struct PacketGeom {
    uint64_t pk_len = 0;  // data bytes of every packet but the last (whole chunks)
    uint32_t upp = 0;     // units per packet but the last
    uint32_t magic = 0, shift = 0;
    uint32_t ptail = 0;   // valid bytes of such a packet's last unit (4096: whole)
    uint32_t lunits = 0;  // units of the last packet (its whole chunks only)
    uint32_t ltail = 0;   // valid bytes of the last packet's last unit
};
// Fills g for npk packets of data_len bytes (the last last_len) with chunks of unit_bpc bytes
// (<= 4096; callers at bpc = R x 4096 pass 4096). False when it does not fit the walk: a non-last
// packet that ends in a short chunk, no unit at all, or 2^31 units or more.
bool packet_geom(uint64_t data_len, uint64_t last_len, uint64_t npk, uint32_t unit_bpc, PacketGeom *g);

struct ChunkLaunch {
    const uint8_t *data;      // device pointer to the first chunk
    uint64_t len;             // bytes
    uint32_t bpc;             // bytes per checksum
    const uint8_t *crc_be;    // verify: stored BE32 words (device)
    uint8_t *out_be;          // compute: BE32 words written here (device)
    unsigned long long *result;  // verify: atomicMax(~first_bad) target (device)
    uint64_t chunk_base;      // added to chunk indices reported in *result
    int check_short_tail;     // 1: tail chunk checked (LocalBlockReader semantics)
    bool overlap_previous = false;  // HDFS3_LAUNCH_OVERLAP_PREVIOUS: AQL packet without barrier bit
    // Packet stream at a constant pitch (PitchWalk, launch_packet_stream): packet i's data at
    // data + i*pitch, its BE32 words at crc_be/out_be + i*pitch; every packet but the last holds
    // geom.pk_len bytes of whole chunks (geom.upp units), the last one last_len <= that many bytes.
    // len is unused; result keys are (packet << 32) | chunk.
    uint64_t pitch = 0;
    uint64_t npk = 0;
    PacketGeom geom;
    uint32_t last_len = 0;
    // pitch mode over independent blocks at constant strides (a [blocks, bytes] tensor and its
    // [blocks, words] tensor): the words' own pitch; 0 = `pitch` (the wire layout of packets)
    uint64_t crc_pitch = 0;
    // Round kernel (launch_wave3 fills these): a wave's round count is kq + (wave < kr), the units of
    // the launch split over its waves on the host, so no wave divides 64-bit values in its prologue.
    uint32_t kq = 0, kr = 0;
    uint32_t lab_seq = 0;  // lab clock stamps only (LabClock): the launch's number
};

// lab clock stamps: launches numbered by the host (kernel argument), see LabClock
inline std::atomic<uint32_t> g_lab_seq{0};

// Packet-descriptor as seen by the device (mirrors hdfs3_pkt_desc).
struct DevPacket {
    uint64_t data_off;
    uint64_t crc_off;
    uint32_t data_len;
    uint32_t reserved;
};

// One independent byte range of a segmented launch (a block of a batch, or one packet's
// data region): device pointers, its 4 KiB units start at global unit unit_begin,
// chunk c of it is reported as key_base + c (packets: packet << 32).
struct DevSegment {
    const uint8_t *data;
    uint8_t *crc;            // verify: stored BE32 words; compute: written here
    uint64_t len;
    uint64_t unit_begin;
    uint64_t key_base;
};

// Units of a segment of len bytes at bpc <= 4096: its whole chunks cut into 4 KiB units, the
// last one partial when the whole chunks end inside a round (PacketGeom); a short last chunk is
// the kernel's one-lane tail
constexpr uint64_t seg_units(uint64_t len, uint32_t bpc) { return (len / bpc * bpc + 4095) / 4096; }

// Fills h_seg for n segments (data/crc/len/key_base already set) and returns the total
// unit count (seg_units); *uniform = units per segment when every segment but the last has
// the same count (direct unit -> segment mapping), else 0 (binary search).
uint64_t plan_segments(DevSegment *h_seg, size_t n, uint32_t bpc, uint64_t *uniform);
// True when the segmented wave kernel can take these segments: bpc in {512..4096},
// every data pointer 16-byte aligned and every CRC pointer 4-byte aligned.
bool segments_fast(const DevSegment *h_seg, size_t n, uint32_t bpc);
// Launches over d_seg (a device copy of a planned h_seg array), or, with h_inline and
// nseg <= 16, over descriptors carried in the kernel arguments (no copy before the kernel).
hipError_t launch_segments(const DevSegment *d_seg, uint32_t nseg, uint64_t units, uint64_t uniform,
                           uint32_t bpc, bool verify, int check_short_tail, unsigned long long *result,
                           const uint32_t *d_tables, const uint32_t *d_fold, int grid_cap, hipStream_t stream,
                           const DevSegment *h_inline = nullptr, uint64_t stride = 0,
                           uint8_t *dense_words = nullptr, const uint32_t *unit_seg = nullptr);
constexpr uint32_t kMaxInlineSegments = 16;

// Packet batch (packets API, block reader, output stream): descriptors in host memory;
// h_stage/d_stage are pinned/device staging for n DevSegments. Uses the segmented wave
// kernel when segments_fast() holds, else the chunk-per-lane packet kernel. Keys are
// (packet << 32 | chunk).
// constant-pitch packet streams (ChunkLaunch::pitch): whether the wave kernel's pitch mode
// takes them (bpc 512..4096 or R x 4096, aligned, every packet but the last whole chunks), and
// its launcher (a.pitch/npk/geom/last_len set)
bool packet_stream_ok(uint64_t data_len, uint64_t last_len, uint64_t npk, uint32_t bpc, const void *data,
                      const void *crc, uint64_t pitch, PacketGeom *geom);
// Compute mode over a stream whose CRC words sit inside each packet (the wire layout: 512 B of
// words per 64 KiB packet, 66 KiB apart) writes 8 MiB per GiB as small regions scattered over
// the arena, interleaved with the read stream: 1 GiB took 213 us against 186 us with the words
// written densely (tools/compute_layout_probe.py, docs/DESIGN_HISTORY.md §4.3). With a WordScratch the words
// go densely into it and one copy kernel scatters them to the packets afterwards.
struct WordScratch {
    uint8_t *d = nullptr;
    uint64_t cap = 0;
    hipEvent_t used = nullptr;  // recorded after the last launch that read the scratch
    void release();
};
// Chunks of R * 4096 bytes (R >= 2; 8 KiB ... 64 KiB and any other multiple of 4096): the round
// kernel computes the CRC of every 4096-byte piece into a ctx-owned scratch (two buffers used in
// turn, so a launch that overlaps its predecessor never writes the words that predecessor's combine
// still reads), then a combine kernel folds each chunk's R piece CRCs (launch_chunks, pieces != null).
// Where a long descriptor list's host-to-device copy runs (round 6): on `side`, beside the launch before
// it, with `stream` waiting for `copied`; in `stream` itself when null or below kSideCopyMinBytes
struct DescCopy {
    hipStream_t side = nullptr;
    hipEvent_t copied = nullptr;
};
constexpr size_t kSideCopyMinBytes = size_t(256) << 10;

struct PieceScratch {
    uint8_t *d[2] = {nullptr, nullptr};
    uint64_t cap[2] = {0, 0};
    hipEvent_t used[2] = {nullptr, nullptr};  // recorded after the combine that read buffer i
    hipStream_t on[2] = {nullptr, nullptr};   // the stream that combine ran on
    unsigned next = 0;
    void release();
};

// word regions at most this long (per packet) take the dense path: 64 KiB = 8 MiB packets at bpc 512
constexpr uint64_t kDenseWordsMaxRegion = 64 * 1024;
// pieces != null: streams at bpc = R * 4096 (R dividing the rounds per packet) take the piece
// CRCs + combine (round 4); without it they return hipErrorNotSupported (the caller's fallback)
hipError_t launch_packet_stream(const ChunkLaunch &a, bool verify, const uint32_t *d_tables, const uint32_t *d_fold,
                                int grid_cap, hipStream_t stream, WordScratch *ws = nullptr,
                                PieceScratch *pieces = nullptr);
// batches of equal blocks (the last may be shorter) of a power-of-two number of whole rounds
// whose data and words sit at two constant strides (blocks of one 2-D tensor): the pitch mode
// with crc_pitch; hipErrorNotSupported = use the segmented kernel
hipError_t launch_strided_blocks(const DevSegment *h_seg, size_t n, uint32_t bpc, bool verify, int check_short_tail,
                                 unsigned long long *result, const uint32_t *d_tables, const uint32_t *d_fold,
                                 int grid_cap, hipStream_t stream, WordScratch *ws = nullptr);
// bad_index != null: every packet is first checked against [0, arena_len) (hipErrorInvalidValue
// and *bad_index = the first one outside). staged != null: set when the launch copies h_stage to the
// device asynchronously (the caller may reuse h_stage only after that copy ran); false when the
// kernel's arguments carried everything (the pitch walk, inline descriptors).
hipError_t launch_packet_batch(const uint8_t *d_arena, const DevPacket *h_pk, size_t n, uint32_t bpc, bool verify,
                               int check_short_tail, unsigned long long *result, DevSegment *h_stage,
                               DevSegment *d_stage, const uint32_t *d_tables, const uint32_t *d_fold, int grid_cap,
                               hipStream_t stream, uint64_t arena_len = 0, size_t *bad_index = nullptr,
                               bool overlap_previous = false, WordScratch *ws = nullptr,
                               PieceScratch *pieces = nullptr, bool *staged = nullptr,
                               const DescCopy *dc = nullptr);

hipError_t launch_chunks(const ChunkLaunch &a, bool verify, const uint32_t *d_tables,
                         const uint32_t *d_fold, int grid_cap, hipStream_t stream,
                         PieceScratch *pieces = nullptr);

hipError_t launch_packets(const uint8_t *d_arena, const DevPacket *d_pk, uint64_t n,
                          uint32_t bpc, bool verify, int check_short_tail,
                          unsigned long long *result, const uint32_t *d_tables, int grid_cap,
                          hipStream_t stream);

// HDFS3_LAB=1 builds the measurement library (libhdfs3_crc_lab.so: tools/, the A/B tests):
// the same production launchers plus a process-wide kernel-variant knob, the kernel
// variants of crc32c_experiments.hip and the read-ceiling kernels. The product library
// (libhdfs3_crc.so) is built with HDFS3_LAB=0: g_variant is the constant 0, so no
// variant, diagnostic or wrong-on-purpose kernel is reachable from it.
#ifndef HDFS3_LAB
#define HDFS3_LAB 0
#endif
#if HDFS3_LAB
void set_variant(int v);
extern int g_variant;
// clock stamps (LabClock): install a device buffer of cap x 4 words; *n_out = stamps in the previous one
hipError_t lab_clock_buffer(unsigned long long *d, unsigned int cap, unsigned int *n_out);
// every wave's stamps (LabClock with a wave buffer): cap x 4 words; *n_out = launches stamped into the
// previous one
hipError_t lab_wave_buffer(unsigned long long *d, unsigned int cap, unsigned int *n_out);
// The A/B variants (crc32c_experiments.hip): variant != 0, bpc with a whole-round kernel.
hipError_t launch_experiment(int variant, const ChunkLaunch &a, bool verify, const uint32_t *tab,
                             const uint32_t *fold, int grid_cap, hipStream_t s);

// Measurement-only kernels (bench/profiling): HBM read ceiling and the CRC
// kernel's access pattern without the table arithmetic.
hipError_t launch_stream_read(const uint8_t *d, uint64_t len, uint32_t *sink, int grid,
                              hipStream_t stream, bool overlap_previous = false);
hipError_t launch_lane_read(const uint8_t *d, uint64_t len, uint32_t bpc, uint32_t *sink,
                            int grid_cap, hipStream_t stream);
#else
constexpr int g_variant = 0;
#endif

}  // namespace hdfs3crc
