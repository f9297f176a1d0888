// Blocking TCP I/O with poll() timeouts: the subset of src/network/TcpSocket.cpp
// (readFully/writeFully, :64-133,334) and BufferedSocketReader.cpp:63-146 (varint
// reads) the checksum path needs. Errors are returned, never thrown.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include <sys/uio.h>

namespace hdfs3crc {
namespace net {

// connect to host:port; returns fd >= 0 or -errno
int connect_tcp(const char *host, int port, int timeout_ms);
// listening socket on 127.0.0.1:port (0 = ephemeral); *bound_port receives the port
int listen_tcp(int port, int *bound_port);
// 0 on success, -errno on failure (-ETIMEDOUT, -ECONNRESET on EOF)
int read_fully(int fd, void *buf, size_t n, int timeout_ms);
// Blocking reads for a socket whose SO_RCVTIMEO was set once (set_recv_timeout): one recv/recvmsg with
// MSG_WAITALL per message when it arrives within the timeout, the way RemoteBlockReader's reading thread
// does it — no poll or setsockopt per call (round 5: the block reader's receiver spent ~4 syscalls per
// packet on them). -ETIMEDOUT when the timeout passes with the message incomplete, -ECONNRESET at EOF.
int set_recv_timeout(int fd, int timeout_ms);
int recv_fully(int fd, void *buf, size_t n);
// na bytes into a, then nb bytes into b (a packet's checksums and data into two places). Round 6
// measured a non-blocking spin before the blocking receive (a receiver polling for data it expects
// instead of sleeping until the sender wakes it): 50 / 200 us of spin took one loopback stream from
// 6.0-7.4 to 3.9-4.5 GiB/s and raised the datanode's CPU per GiB by half (profiles/r06/r6g_*): a
// receiver that takes each packet in one MSG_WAITALL receive is the cheapest for the sender too.
int recv_fully2(int fd, void *a, size_t na, void *b, size_t nb);
// n pieces in order, as few MSG_WAITALL receives as the data allows (the block reader takes a packet's
// checksums, its data and the NEXT packet's fixed 31-byte header in one: one receive per packet)
int recv_fully_iov(int fd, iovec *v, int n);
int write_fully(int fd, const void *buf, size_t n, int timeout_ms);
// protobuf varint32 length prefix, as BufferedSocketReader::readVarint32
int read_varint32(int fd, uint32_t *out, int timeout_ms);
// read a varint-length-prefixed message (bounded by max_len, RemoteBlockReader.cpp:116)
int read_delimited(int fd, std::string &out, size_t max_len, int timeout_ms);
int write_delimited(int fd, const std::string &msg, int timeout_ms);
// poll for readability: 1 readable (or EOF/error pending), 0 not within timeout_ms, -errno
int readable(int fd, int timeout_ms);
void close_fd(int fd);

}  // namespace net
}  // namespace hdfs3crc
