// Probe for the short-circuit reader (docs/DESIGN_HISTORY.md §5.1): can a block file's page-cache pages be
// DMA'd to the GPU directly? mmap the file, hipHostRegister the mapping (pins the page-cache
// pages), time the registration, an H2D copy from it, and the unregister; compare with pread
// into pinned memory + H2D, and with a plain read() of the file.
// Build: hipcc -O2 --offload-arch=gfx950 tools/mmap_register_probe.cpp -o tools/mmap_register_probe
// Run:   tools/mmap_register_probe <file of N MiB>   (writes one JSON line per measurement)
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define OK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));       \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const int fd = open(argv[1], O_RDONLY);
    if (fd < 0) return 3;
    struct stat st;
    fstat(fd, &st);
    const size_t n = size_t(st.st_size);
    std::vector<char> user(n);
    void *d = nullptr, *pinned = nullptr;
    OK(hipMalloc(&d, n));
    OK(hipHostMalloc(&pinned, n, hipHostMallocDefault));
    hipStream_t s;
    OK(hipStreamCreate(&s));
    for (int rep = 0; rep < 3; ++rep) {
        // plain read() of the whole file (page cache warm after rep 0)
        double t0 = now();
        size_t got = 0;
        while (got < n) {
            const ssize_t r = pread(fd, user.data() + got, n - got, off_t(got));
            if (r <= 0) return 4;
            got += size_t(r);
        }
        const double t_read = now() - t0;
        // pread into pinned + H2D
        t0 = now();
        got = 0;
        while (got < n) {
            const ssize_t r = pread(fd, static_cast<char *>(pinned) + got, n - got, off_t(got));
            if (r <= 0) return 5;
            got += size_t(r);
        }
        const double t_pread_pinned = now() - t0;
        double t1 = now();
        OK(hipMemcpyAsync(d, pinned, n, hipMemcpyHostToDevice, s));
        OK(hipStreamSynchronize(s));
        const double t_h2d_pinned = now() - t1;
        // mmap + register + H2D + copy-out from the mapping + unregister
        t0 = now();
        void *m = mmap(nullptr, n, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
        if (m == MAP_FAILED) return 6;
        const double t_mmap = now() - t0;
        t1 = now();
        const hipError_t reg = hipHostRegister(m, n, hipHostRegisterReadOnly);
        const double t_reg = now() - t1;
        double t_h2d_mapped = -1, t_unreg = -1;
        if (reg == hipSuccess) {
            t1 = now();
            OK(hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, s));
            OK(hipStreamSynchronize(s));
            t_h2d_mapped = now() - t1;
        }
        t1 = now();
        std::memcpy(user.data(), m, n);
        const double t_copy_from_map = now() - t1;
        if (reg == hipSuccess) {
            t1 = now();
            OK(hipHostUnregister(m));
            t_unreg = now() - t1;
        }
        munmap(m, n);
        const double gib = double(n) / double(1u << 30);
        std::printf("{\"probe\": \"mmap_register\", \"rep\": %d, \"bytes\": %zu, \"read_GiBps\": %.2f, "
                    "\"pread_pinned_GiBps\": %.2f, \"h2d_pinned_GiBps\": %.2f, \"mmap_populate_ms\": %.3f, "
                    "\"register\": \"%s\", \"register_ms\": %.3f, \"h2d_mapped_GiBps\": %.2f, \"unregister_ms\": %.3f, "
                    "\"copy_from_map_GiBps\": %.2f}\n",
                    rep, n, gib / t_read, gib / t_pread_pinned, gib / t_h2d_pinned, t_mmap * 1e3,
                    hipGetErrorString(reg), t_reg * 1e3, t_h2d_mapped > 0 ? gib / t_h2d_mapped : -1.0,
                    t_unreg * 1e3, gib / t_copy_from_map);
        std::fflush(stdout);
    }
    // registration cost by piece size over one mapping (page cache warm)
    void *m = mmap(nullptr, n, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
    if (m == MAP_FAILED) return 7;
    for (size_t piece : {size_t(1) << 20, size_t(4) << 20, size_t(16) << 20, size_t(32) << 20, n}) {
        double t_reg = 0, t_unreg = 0;
        size_t k = 0;
        for (size_t off = 0; off + piece <= n; off += piece, ++k) {
            double t1 = now();
            OK(hipHostRegister(static_cast<char *>(m) + off, piece, hipHostRegisterReadOnly));
            t_reg += now() - t1;
            t1 = now();
            OK(hipHostUnregister(static_cast<char *>(m) + off));
            t_unreg += now() - t1;
        }
        std::printf("{\"probe\": \"register_pieces\", \"piece_mib\": %zu, \"pieces\": %zu, \"register_ms_per_piece\": %.4f, "
                    "\"register_GiBps\": %.2f, \"unregister_ms_per_piece\": %.4f}\n",
                    piece >> 20, k, t_reg * 1e3 / k, double(piece * k) / (1u << 30) / t_reg, t_unreg * 1e3 / k);
    }
    munmap(m, n);
    return 0;
}
