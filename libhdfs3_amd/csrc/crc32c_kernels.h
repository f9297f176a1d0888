// Internal launch interface of the gfx950 CRC32C kernels (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace hdfs3crc {

// Workgroup geometry: the bank-replicated slice-table image takes 128 KiB of
// the CU's 160 KiB LDS, so one workgroup owns a CU; 1024 threads = 16 waves
// (4 per SIMD) keep the CU's memory pipe and LDS busy.
constexpr int kBlockThreads = 1024;

struct ChunkLaunch {
    const uint8_t *data;      // device pointer to the first chunk
    uint64_t len;             // bytes
    uint32_t bpc;             // bytes per checksum
    const uint8_t *crc_be;    // verify: stored BE32 words (device)
    uint8_t *out_be;          // compute: BE32 words written here (device)
    unsigned long long *result;  // verify: atomicMax(~first_bad) target (device)
    uint64_t chunk_base;      // added to chunk indices reported in *result
    int check_short_tail;     // 1: tail chunk checked (LocalBlockReader semantics)
    uint64_t *trace = nullptr;  // diagnostic variant 13 only: 4 s_memrealtime stamps per wave
};

// Packet-descriptor as seen by the device (mirrors hdfs3_pkt_desc).
struct DevPacket {
    uint64_t data_off;
    uint64_t crc_off;
    uint32_t data_len;
    uint32_t reserved;
};

hipError_t launch_chunks(const ChunkLaunch &a, bool verify, const uint32_t *d_tables,
                         const uint32_t *d_fold, int grid_cap, hipStream_t stream);

hipError_t launch_packets(const uint8_t *d_arena, const DevPacket *d_pk, uint64_t n,
                          uint32_t bpc, bool verify, int check_short_tail,
                          unsigned long long *result, const uint32_t *d_tables, int grid_cap,
                          hipStream_t stream);

// Measurement knob: selects kernel variants for in-process A/B (0 = production).
void set_variant(int v);
void set_trace(uint64_t *d_trace);  // buffer for variant 13 (4 x u64 per wave)

// Measurement-only kernels (bench/profiling): HBM read ceiling and the CRC
// kernel's access pattern without the table arithmetic.
hipError_t launch_stream_read(const uint8_t *d, uint64_t len, uint32_t *sink, int grid,
                              hipStream_t stream);
hipError_t launch_lane_read(const uint8_t *d, uint64_t len, uint32_t bpc, uint32_t *sink,
                            int grid_cap, hipStream_t stream);

}  // namespace hdfs3crc
