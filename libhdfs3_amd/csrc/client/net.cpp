#include "net.h"

#include <arpa/inet.h>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/time.h>
#include <unistd.h>

namespace hdfs3crc {
namespace net {

static int wait_fd(int fd, short events, int timeout_ms) {
    pollfd p{fd, events, 0};
    for (;;) {
        const int rc = poll(&p, 1, timeout_ms);
        if (rc > 0) return 0;
        if (rc == 0) return -ETIMEDOUT;
        if (errno != EINTR) return -errno;
    }
}

int readable(int fd, int timeout_ms) {
    const int rc = wait_fd(fd, POLLIN, timeout_ms);
    return rc == 0 ? 1 : rc == -ETIMEDOUT ? 0 : rc;
}

int connect_tcp(const char *host, int port, int timeout_ms) {
    addrinfo hints{};
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo *res = nullptr;
    char portstr[16];
    snprintf(portstr, sizeof(portstr), "%d", port);
    if (getaddrinfo(host, portstr, &hints, &res) != 0 || !res) return -EHOSTUNREACH;
    const int fd = socket(res->ai_family, SOCK_STREAM, 0);
    if (fd < 0) {
        freeaddrinfo(res);
        return -errno;
    }
    const int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));  // as RemoteBlockReader.cpp:100
    const int flags = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, flags | O_NONBLOCK);
    int rc = connect(fd, res->ai_addr, res->ai_addrlen);
    freeaddrinfo(res);
    if (rc < 0 && errno == EINPROGRESS) {
        rc = wait_fd(fd, POLLOUT, timeout_ms);
        if (rc == 0) {
            int err = 0;
            socklen_t len = sizeof(err);
            getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
            rc = err ? -err : 0;
        }
    } else if (rc < 0) {
        rc = -errno;
    }
    if (rc < 0) {
        ::close(fd);
        return rc;
    }
    fcntl(fd, F_SETFL, flags);
    return fd;
}

int listen_tcp(int port, int *bound_port) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return -errno;
    const int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons(uint16_t(port));
    if (bind(fd, reinterpret_cast<sockaddr *>(&a), sizeof(a)) < 0 || listen(fd, 16) < 0) {
        const int e = -errno;
        ::close(fd);
        return e;
    }
    socklen_t len = sizeof(a);
    getsockname(fd, reinterpret_cast<sockaddr *>(&a), &len);
    if (bound_port) *bound_port = ntohs(a.sin_port);
    return fd;
}

// Reads of at least this many bytes that find nothing buffered wait for their whole remainder in one
// blocking recv (MSG_WAITALL under SO_RCVTIMEO): a 64 KiB packet payload arriving as many TCP segments
// then costs one wake-up of the reading thread instead of a poll + recv per segment (round 5)
constexpr size_t kWaitAllMin = 4096;

int read_fully(int fd, void *buf, size_t n, int timeout_ms) {
    char *p = static_cast<char *>(buf);
    while (n) {
        // what is already buffered first: no poll when the data is there
        const ssize_t r = ::recv(fd, p, n, MSG_DONTWAIT);
        if (r > 0) {
            p += r;
            n -= size_t(r);
            continue;
        }
        if (r == 0) return -ECONNRESET;  // peer closed before the message was complete
        if (errno == EINTR) continue;
        if (errno != EAGAIN && errno != EWOULDBLOCK) return -errno;
        if (n >= kWaitAllMin && timeout_ms > 0) {
            // the socket's SO_RCVTIMEO is this call's timeout (the connection's one timeout: callers
            // pass the same value on every read of a socket)
            timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
            if (setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv)) == 0) {
                const ssize_t w = ::recv(fd, p, n, MSG_WAITALL);
                if (w > 0) {  // all of it, or what arrived before the timeout / a signal
                    p += w;
                    n -= size_t(w);
                    continue;
                }
                if (w == 0) return -ECONNRESET;
                if (errno == EINTR) continue;
                // EAGAIN with nothing read: SO_RCVTIMEO expired, the whole timeout has passed (ADVICE
                // r5: waiting again in poll doubled it)
                if (errno == EAGAIN || errno == EWOULDBLOCK) return -ETIMEDOUT;
                return -errno;
            }
        }
        // poll: a blocking recv without SO_RCVTIMEO would ignore the timeout
        if (const int rc = wait_fd(fd, POLLIN, timeout_ms)) return rc;
    }
    return 0;
}

int set_recv_timeout(int fd, int timeout_ms) {
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    return setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv)) == 0 ? 0 : -errno;
}

int recv_fully_iov(int fd, iovec *v, int n) {
    int first = 0;
    while (first < n && v[first].iov_len == 0) ++first;
    while (first < n) {
        msghdr m{};
        m.msg_iov = v + first;
        m.msg_iovlen = size_t(n - first);
        const ssize_t r = ::recvmsg(fd, &m, MSG_WAITALL);
        if (r < 0) {
            if (errno == EINTR) continue;
            return errno == EAGAIN || errno == EWOULDBLOCK ? -ETIMEDOUT : -errno;
        }
        if (r == 0) return -ECONNRESET;
        size_t got = size_t(r);
        while (got && first < n) {
            const size_t take = got < v[first].iov_len ? got : v[first].iov_len;
            v[first].iov_base = static_cast<char *>(v[first].iov_base) + take;
            v[first].iov_len -= take;
            got -= take;
            if (v[first].iov_len == 0) ++first;
        }
        while (first < n && v[first].iov_len == 0) ++first;
    }
    return 0;
}

int recv_fully2(int fd, void *a, size_t na, void *b, size_t nb) {
    iovec v[2] = {{a, na}, {b, nb}};
    return recv_fully_iov(fd, v, 2);
}

int recv_fully(int fd, void *buf, size_t n) { return recv_fully2(fd, buf, n, nullptr, 0); }

int write_fully(int fd, const void *buf, size_t n, int timeout_ms) {
    const char *p = static_cast<const char *>(buf);
    while (n) {
        // send first: poll only when the socket's buffer is full (round 5; a poll per send before)
        const ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL | MSG_DONTWAIT);
        if (r > 0) {
            p += r;
            n -= size_t(r);
        } else if (r < 0 && errno == EINTR) {
            continue;
        } else if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
            if (const int rc = wait_fd(fd, POLLOUT, timeout_ms)) return rc;
        } else {
            return r < 0 ? -errno : -EIO;
        }
    }
    return 0;
}

int read_varint32(int fd, uint32_t *out, int timeout_ms) {
    uint32_t v = 0;
    for (int shift = 0; shift < 35; shift += 7) {
        uint8_t b;
        if (const int rc = read_fully(fd, &b, 1, timeout_ms)) return rc;
        v |= uint32_t(b & 0x7F) << shift;
        if (!(b & 0x80)) {
            *out = v;
            return 0;
        }
    }
    return -EPROTO;
}

int read_delimited(int fd, std::string &out, size_t max_len, int timeout_ms) {
    uint32_t n = 0;
    if (const int rc = read_varint32(fd, &n, timeout_ms)) return rc;
    if (n == 0 || n > max_len) return -EPROTO;
    out.resize(n);
    return read_fully(fd, &out[0], n, timeout_ms);
}

int write_delimited(int fd, const std::string &msg, int timeout_ms) {
    std::string buf;
    uint64_t v = msg.size();
    while (v >= 0x80) {
        buf.push_back(char(uint8_t(v) | 0x80));
        v >>= 7;
    }
    buf.push_back(char(v));
    buf += msg;
    return write_fully(fd, buf.data(), buf.size(), timeout_ms);
}

void close_fd(int fd) {
    if (fd >= 0) ::close(fd);
}

}  // namespace net
}  // namespace hdfs3crc
