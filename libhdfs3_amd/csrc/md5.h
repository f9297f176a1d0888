// MD5 (RFC 1321), host side. Used only for the block checksum ("MD5 of CRC32",
// DataTransferProtocolSender.h:113, OpBlockChecksumResponseProto datatransfer.proto:222-227):
// the digest runs over the block's big-endian CRC words, 4 bytes per chunk, which is
// 1/128 of the block at 512 B chunks. MD5 is a serial chain (Merkle-Damgard), so it is
// not GPU work; the CRC words it digests are computed on the GPU.
#pragma once

#include <cstddef>
#include <cstdint>

namespace hdfs3crc {

struct Md5 {
    uint32_t h[4];
    uint64_t total = 0;       // bytes absorbed
    uint8_t buf[64];
    size_t fill = 0;

    Md5();
    void update(const void *p, size_t n);
    void finish(uint8_t out[16]);
};

}  // namespace hdfs3crc
