// Wire formats on the checksum path, hand-encoded (no protobuf runtime in this image).
//
//  * PacketHeader (src/client/PacketHeader.cpp:38-123, datatransfer.proto:143-150):
//      BE32 packetLen | BE16 protoLen | PacketHeaderProto
//    with PacketHeaderProto = {1: sfixed64 offsetInBlock, 2: sfixed64 seqno,
//    3: bool lastPacketInBlock, 4: sfixed32 dataLen, [5: bool syncBlock]}. All fields
//    fixed-width, so the header the reference writes is 31 bytes (CalcPkgHeaderSize).
//  * Data-transfer request framing (DataTransferProtocolSender.cpp:42-57):
//      BE16 version (28) | u8 op (READ_BLOCK = 81) | varint len | OpReadBlockProto
//  * Responses: varint len | BlockOpResponseProto (RemoteBlockReader.cpp:112-203), and
//    the client's final varint len | ClientReadStatusProto (RemoteBlockReader.cpp:289-304).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace hdfs3crc {
namespace wire {

constexpr int kDataTransferVersion = 28;   // DataTransferProtocolSender.h:38
constexpr int kOpWriteBlock = 80;          // DataTransferProtocolSender.h:44
constexpr int kOpReadBlock = 81;           // DataTransferProtocolSender.h:45
constexpr int kOpBlockChecksum = 85;       // DataTransferProtocolSender.h:49
constexpr int kPacketHeaderSize = 31;      // PacketHeader::CalcPkgHeaderSize with all fields set

enum Status : int {                        // datatransfer.proto:152-166
    kSuccess = 0,
    kError = 1,
    kErrorChecksum = 2,
    kErrorInvalid = 3,
    kChecksumOk = 6,
};
enum ChecksumType : int { kChecksumNull = 0, kChecksumCrc32 = 1, kChecksumCrc32c = 2 };  // hdfs.proto:262-266

// ---- protobuf primitives ------------------------------------------------------
void put_varint(std::string &out, uint64_t v);
void put_tag(std::string &out, int field, int wiretype);
void put_fixed64(std::string &out, uint64_t v);
void put_fixed32(std::string &out, uint32_t v);
void put_bytes(std::string &out, int field, const std::string &s);
void put_uint(std::string &out, int field, uint64_t v);

// Minimal reader over a protobuf message; unknown fields are skipped.
struct Reader {
    const uint8_t *p, *end;
    bool ok = true;
    Reader(const void *b, size_t n) : p(static_cast<const uint8_t *>(b)), end(p + n) {}
    bool more() const { return ok && p < end; }
    uint64_t varint();
    uint64_t fixed64();
    uint32_t fixed32();
    std::string bytes();
    void skip(int wiretype);
};

// ---- PacketHeader -------------------------------------------------------------
struct PacketHeader {
    int32_t packet_len = 0;        // dataLen + checksum bytes + 4 (Packet.cpp:146-147)
    int64_t offset_in_block = 0;
    int64_t seqno = 0;
    bool last_packet_in_block = false;
    int32_t data_len = 0;
    bool sync_block = false;       // never written by the client (Packet.cpp:146-148)

    // 31 bytes: BE32 packetLen, BE16 protoLen = 25, proto fields 1..4
    void encode(uint8_t out[kPacketHeaderSize]) const;
    // PacketHeader::readFields (PacketHeader.cpp:100-117); false on malformed input
    bool decode(const uint8_t *buf, size_t n);
    // PacketHeader::sanityCheck (PacketHeader.cpp:72-86)
    bool sanity_check(int64_t last_seqno) const;
};

// ---- requests / responses -----------------------------------------------------
struct ExtendedBlock {             // hdfs.proto:38-44
    std::string pool_id;
    uint64_t block_id = 0;
    uint64_t generation_stamp = 0;
    uint64_t num_bytes = 0;
};

struct ReadBlockRequest {          // OpReadBlockProto, datatransfer.proto:63-69
    ExtendedBlock block;
    std::string client_name;
    uint64_t offset = 0;
    uint64_t len = 0;
    bool send_checksums = true;
};
// full framed request: version | op | varint len | proto
std::string encode_read_block(const ReadBlockRequest &r);
// parse the proto part of a READ_BLOCK request (datanode side)
bool decode_read_block(const void *proto, size_t n, ReadBlockRequest &out);

struct BlockChecksumResponse {     // OpBlockChecksumResponseProto, datatransfer.proto:222-227
    uint32_t bytes_per_crc = 0;
    uint64_t crc_per_block = 0;
    std::string md5;               // 16 bytes: MD5 of the block's BE CRC words
    int crc_type = -1;             // optional ChecksumTypeProto; -1 when absent
};

// OP_BLOCK_CHECKSUM request (DataTransferProtocolSender::blockChecksum, a TODO in the
// reference at DataTransferProtocolSender.cpp:169-180): version | op 85 | varint len |
// OpBlockChecksumProto {1: BaseHeaderProto {1: block, 2: token}} (datatransfer.proto:128-130)
std::string encode_block_checksum(const ExtendedBlock &block);
bool decode_block_checksum(const void *proto, size_t n, ExtendedBlock &out);

struct BlockOpResponse {           // BlockOpResponseProto, datatransfer.proto:189-209
    int status = kSuccess;
    std::string first_bad_link;           // field 2 (WRITE_BLOCK setup replies, Pipeline.cpp:562)
    bool has_checksum_response = false;   // field 3 (OP_BLOCK_CHECKSUM replies)
    BlockChecksumResponse checksum_response;
    bool has_checksum_info = false;
    int checksum_type = kChecksumCrc32c;
    uint32_t bytes_per_checksum = 512;
    uint64_t chunk_offset = 0;
    std::string message;
};
std::string encode_block_op_response(const BlockOpResponse &r);   // proto only
bool decode_block_op_response(const void *proto, size_t n, BlockOpResponse &out);

// OP_WRITE_BLOCK (DataTransferProtocolSender::writeBlock, DataTransferProtocolSender.cpp:
// 125-150): version | op 80 | varint len | OpWriteBlockProto (datatransfer.proto:77-111)
struct DatanodeAddr {              // DatanodeInfoProto.id (hdfs.proto:49-60,72-90): the fields
    std::string ip_addr;           // BuildNodeInfo sets (DataTransferProtocolSender.cpp:80-90)
    std::string host_name;
    std::string uuid;
    uint32_t xfer_port = 0;
    uint32_t info_port = 0;
    uint32_t ipc_port = 0;
    std::string location;          // DatanodeInfoProto.location (field 8), set by BuildNodeInfo
};
// BlockConstructionStage (Pipeline.h:50-70)
enum BlockConstructionStage : int {
    kPipelineSetupAppend = 0,
    kDataStreaming = 2,
    kPipelineClose = 4,
    kPipelineSetupCreate = 6
};
struct WriteBlockRequest {
    ExtendedBlock block;
    std::string client_name;
    std::vector<DatanodeAddr> targets;  // the downstream nodes (nodes[1..], Pipeline.cpp:539-543)
    int stage = kPipelineSetupCreate;
    uint32_t pipeline_size = 0;         // targets.size() (DataTransferProtocolSender.cpp:135)
    uint64_t min_bytes_rcvd = 0;
    uint64_t max_bytes_rcvd = 0;
    uint64_t latest_generation_stamp = 0;
    int checksum_type = kChecksumCrc32c;
    uint32_t bytes_per_checksum = 512;
};
std::string encode_write_block(const WriteBlockRequest &r);
bool decode_write_block(const void *proto, size_t n, WriteBlockRequest &out);

// PipelineAckProto {1: sint64 seqno, 2: repeated Status, 3: uint64 downstreamAckTimeNanos}
// (datatransfer.proto:168-172), varint-length-delimited on the wire (Pipeline.cpp:724-740)
constexpr int64_t kHeartbeatSeqno = -1;   // Pipeline.h HEART_BEAT_SEQNO
struct PipelineAck {
    int64_t seqno = 0;
    std::vector<int> status;            // one per node, upstream first
    uint64_t downstream_ack_time_nanos = 0;
    bool success() const {              // PipelineAck::isSuccess (PipelineAck.h:63-73)
        for (int s : status)
            if (s != kSuccess) return false;
        return true;
    }
};
std::string encode_pipeline_ack(const PipelineAck &a);   // proto only
bool decode_pipeline_ack(const void *proto, size_t n, PipelineAck &out);

std::string encode_client_read_status(int status);                // proto only
bool decode_client_read_status(const void *proto, size_t n, int &status);

// big-endian helpers (src/common/BigEndian.h:43-59)
inline uint32_t rd_be32(const uint8_t *p) {
    return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}
inline uint16_t rd_be16(const uint8_t *p) { return uint16_t((p[0] << 8) | p[1]); }
inline void wr_be32(uint8_t *p, uint32_t v) {
    p[0] = uint8_t(v >> 24); p[1] = uint8_t(v >> 16); p[2] = uint8_t(v >> 8); p[3] = uint8_t(v);
}
inline void wr_be16(uint8_t *p, uint16_t v) { p[0] = uint8_t(v >> 8); p[1] = uint8_t(v); }

}  // namespace wire
}  // namespace hdfs3crc
