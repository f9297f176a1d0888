// CPU test of csrc/client/net.cpp's reads (tests/test_wire_sanitized.py builds it under ASan/UBSan):
// a writer thread sends a byte stream in random-sized pieces with random pauses over a socketpair;
// the reader takes it apart with read_fully and recv_fully2 (scatter into two buffers, the block
// reader's [checksums][data] read) in random-sized requests, and every byte must land where expected.
// Also: EOF mid-message is -ECONNRESET, and a silent peer times out as -ETIMEDOUT once, for short and
// for long reads (a read of >= 4 KiB waits in one MSG_WAITALL recv under SO_RCVTIMEO: ADVICE r5).
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "client/net.h"

using namespace hdfs3crc;

static int fail(const char *what) {
    std::printf("FAIL %s\n", what);
    return 1;
}

int main() {
    std::mt19937_64 rng(12345);
    const size_t total = 24u << 20;
    std::vector<unsigned char> src(total);
    for (auto &c : src) c = static_cast<unsigned char>(rng());
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv)) return fail("socketpair");
    std::thread writer([&] {
        std::mt19937_64 r(777);
        size_t off = 0;
        while (off < total) {
            size_t n = 1 + r() % 200000;
            if (n > total - off) n = total - off;
            if (net::write_fully(sv[1], src.data() + off, n, 10000)) break;
            off += n;
            if (r() % 8 == 0) std::this_thread::sleep_for(std::chrono::microseconds(r() % 300));
        }
    });
    if (net::set_recv_timeout(sv[0], 10000)) return fail("set_recv_timeout");
    std::vector<unsigned char> a(70000), b(300000);
    size_t off = 0;
    while (off < total) {
        const size_t left = total - off;
        const unsigned pick = unsigned(rng() % 3);
        if (pick == 2) {  // the block reader's receive: blocking WAITALL under SO_RCVTIMEO
            size_t na = rng() % 600, nb = rng() % 250000;
            if (na > left) na = left;
            if (nb > left - na) nb = left - na;
            if (net::recv_fully2(sv[0], a.data(), na, b.data(), nb)) return fail("recv_fully2");
            if (std::memcmp(a.data(), src.data() + off, na) || std::memcmp(b.data(), src.data() + off + na, nb))
                return fail("recv_fully2 bytes");
            off += na + nb;
        } else if (pick < 2) {
            size_t n = 1 + rng() % 250000;
            if (n > left) n = left;
            if (net::read_fully(sv[0], b.data(), n, 10000)) return fail("read_fully");
            if (std::memcmp(b.data(), src.data() + off, n)) return fail("read_fully bytes");
            off += n;
        }
    }
    writer.join();
    // a silent peer: both reads time out
    if (net::read_fully(sv[0], b.data(), 10, 200) != -ETIMEDOUT) return fail("read_fully timeout");
    {  // a long read times out after one timeout, not two
        const auto t0 = std::chrono::steady_clock::now();
        if (net::read_fully(sv[0], b.data(), 100000, 200) != -ETIMEDOUT) return fail("read_fully long timeout");
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms < 150 || ms > 350) {
            std::printf("long read timed out after %.0f ms\n", ms);
            return fail("read_fully long timeout duration");
        }
    }
    if (net::set_recv_timeout(sv[0], 200)) return fail("set_recv_timeout 200");
    if (net::recv_fully(sv[0], b.data(), 10) != -ETIMEDOUT) return fail("recv_fully timeout");
    if (net::recv_fully2(sv[0], a.data(), 31, b.data(), 65536) != -ETIMEDOUT) return fail("recv_fully2 timeout");
    // EOF in the middle of a message
    if (net::write_fully(sv[1], src.data(), 5000, 1000)) return fail("write");
    shutdown(sv[1], SHUT_WR);
    if (net::read_fully(sv[0], b.data(), 11000, 1000) != -ECONNRESET) return fail("read_fully eof");
    close(sv[0]);
    close(sv[1]);
    std::printf("net reads ok\n");
    return 0;
}
