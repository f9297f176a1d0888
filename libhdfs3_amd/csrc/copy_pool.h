// Internal: a small process-wide pool of host threads for the large CPU copies around the GPU
// work — staging pageable caller buffers into pinned memory (hdfs3_crc32c_verify/compute),
// copying verified windows out to the caller and preading block files (local reader). One
// thread copies ~11-28 GiB/s depending on the memory involved, below the PCIe rate these
// paths feed, so copies of 2 MiB or more are split over the caller and the helpers (3;
// HDFS3_COPY_HELPERS=n sets n, 0 copies on the calling thread only). A caller always copies
// its own first piece and then takes queued pieces itself, so concurrent callers (a local
// reader's loader and its consumer) share the helpers without waiting on each other. The pool
// is leaked on purpose: its threads block on its condition variable until the process exits.
// Not installed.
#pragma once

#include <unistd.h>

#include <cstdlib>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#if defined(__x86_64__) || defined(__i386__)
#include <immintrin.h>
#define HDFS3_COPY_NT_AVAILABLE 1
#else
#define HDFS3_COPY_NT_AVAILABLE 0
#endif

namespace hdfs3crc {

// Copies with streaming (non-temporal) stores: the destination lines are written without being read
// first, so a DRAM-bound copy moves 2 bytes per byte instead of 3 (round 4 measurement knob,
// HDFS3_COPY_NT=1; the default is memcpy). Destination aligned to 32 B, 128 B per iteration. x86 only:
// elsewhere the knob is ignored and every copy is memcpy.
#if HDFS3_COPY_NT_AVAILABLE
__attribute__((target("avx2"))) inline void memcpy_stream(uint8_t *dst, const uint8_t *src, size_t n) {
    size_t head = (32 - (reinterpret_cast<uintptr_t>(dst) & 31)) & 31;
    if (head > n) head = n;
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 64));
        const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(src + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(dst + i + 96), d);
    }
    std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();  // the streaming stores are weakly ordered: visible before the piece is reported done
}
#else
inline void memcpy_stream(uint8_t *dst, const uint8_t *src, size_t n) { std::memcpy(dst, src, n); }
#endif

inline int pread_fully(int fd, void *buf, size_t n, int64_t off) {
    uint8_t *p = static_cast<uint8_t *>(buf);
    while (n) {
        const ssize_t r = ::pread(fd, p, n, off);
        if (r < 0) {
            if (errno == EINTR) continue;
            return -errno;
        }
        if (r == 0) return -EIO;  // file shorter than the block / meta says
        p += r;
        n -= size_t(r);
        off += r;
    }
    return 0;
}

class CopyPool {
  public:
    static CopyPool &get() {
        static CopyPool *p = new CopyPool();
        return *p;
    }
    void copy(void *dst, const void *src, size_t n) {
        split(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), -1, 0, n);
    }
    // pread of [off, off + n) of fd into dst, in parallel pieces; 0 or -errno
    int pread(int fd, void *dst, size_t n, int64_t off) { return split(static_cast<uint8_t *>(dst), nullptr, fd, off, n); }
  private:
    static constexpr size_t kMin = 2u << 20;
    static constexpr size_t kNtMin = 256u << 10;
    size_t helpers_ = 3;
    bool nt_ = false;
    struct Job {
        uint8_t *dst = nullptr;
        const uint8_t *src = nullptr;  // memcpy source, or null: pread from fd at off
        int fd = -1;
        int64_t off = 0;
        size_t n = 0;
        std::atomic<int> *pending = nullptr;
        std::atomic<int> *err = nullptr;
    };
    void run(const Job &j) {
        if (j.src) {
            if (nt_ && j.n >= kNtMin) memcpy_stream(j.dst, j.src, j.n);
            else std::memcpy(j.dst, j.src, j.n);
        } else if (int rc = pread_fully(j.fd, j.dst, j.n, j.off)) {
            j.err->store(rc, std::memory_order_relaxed);
        }
        // the last piece of a split wakes its waiter (after this, the split's counters may be gone:
        // only pool members are touched)
        if (j.pending->fetch_sub(1, std::memory_order_acq_rel) == 1) {
            std::lock_guard<std::mutex> lk(done_mu_);
            done_cv_.notify_all();
        }
    }
    // help with pieces no helper has taken yet, then wait for the rest: a short spin (the pieces
    // are equal, so they usually finish together), then block on the pool's completion variable
    // instead of burning a core per waiting caller
    void help_and_wait(std::atomic<int> &pending) {
        for (;;) {
            Job j;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (jobs_.empty()) break;
                j = jobs_.back();
                jobs_.pop_back();
            }
            run(j);
        }
        for (int i = 0; i < 64 && pending.load(std::memory_order_acquire) != 0; ++i) std::this_thread::yield();
        if (pending.load(std::memory_order_acquire) == 0) return;
        std::unique_lock<std::mutex> lk(done_mu_);
        done_cv_.wait(lk, [&] { return pending.load(std::memory_order_acquire) == 0; });
    }
    int split(uint8_t *dst, const uint8_t *src, int fd, int64_t foff, size_t n) {
        std::atomic<int> pending{0}, err{0};
        if (n < kMin || helpers_ == 0) {
            pending.fetch_add(1, std::memory_order_relaxed);
            run(Job{dst, src, fd, foff, n, &pending, &err});
            return err.load();
        }
        const size_t parts = helpers_ + 1;
        // ceil(n / parts), rounded up to 4 KiB: the parts pieces cover all n bytes
        const size_t piece = ((n + parts - 1) / parts + 4095) & ~size_t(4095);
        size_t off = piece;
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (size_t i = 1; i < parts && off < n; ++i, off += piece) {
                jobs_.push_back(Job{dst + off, src ? src + off : nullptr, fd, foff + int64_t(off), std::min(piece, n - off),
                                    &pending, &err});
                pending.fetch_add(1, std::memory_order_relaxed);
            }
        }
        cv_.notify_all();
        pending.fetch_add(1, std::memory_order_relaxed);
        run(Job{dst, src, fd, foff, std::min(piece, n), &pending, &err});
        help_and_wait(pending);
        return err.load();
    }
    CopyPool() {
        if (const char *e = getenv("HDFS3_COPY_HELPERS")) helpers_ = size_t(std::min(std::max(atoi(e), 0), 15));
#if HDFS3_COPY_NT_AVAILABLE
        if (const char *e = getenv("HDFS3_COPY_NT")) nt_ = e[0] == '1' && __builtin_cpu_supports("avx2");
#endif
        for (size_t i = 0; i < helpers_; ++i)
            std::thread([this] {
                for (;;) {
                    Job j;
                    {
                        std::unique_lock<std::mutex> lk(mu_);
                        cv_.wait(lk, [this] { return !jobs_.empty(); });
                        j = jobs_.front();
                        jobs_.pop_front();
                    }
                    run(j);
                }
            }).detach();
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Job> jobs_;
    std::mutex done_mu_;
    std::condition_variable done_cv_;
};

}  // namespace hdfs3crc
