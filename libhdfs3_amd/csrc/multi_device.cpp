// Independent HDFS blocks sharded over several GPUs (include/hdfs3_crc.h, hdfs3_multi_*):
// block b -> devices[b % n], one context, HIP stream and host worker thread per device, no
// collective and no cross-device traffic (BASELINE.json configs[3]).
//
// The reference verifies blocks one at a time on the reading thread
// (InputStreamImpl::readOneBlock, InputStreamImpl.cpp:616-708, and RemoteBlockReader::
// verifyChecksum per packet, RemoteBlockReader.cpp:306-326); its only parallelism is one
// stream per caller thread. Here every device works through its share of the blocks at the
// same time, and a call returns when the slowest device is done.
#include "hdfs3_crc.h"

#include <hip/hip_runtime.h>

#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "ctx.h"
#include "numa.h"

using hdfs3crc::fail;

namespace {

// One device: its ctx, a per-block result array (device + pinned host) and a worker thread
// that runs one job at a time with that device current.
struct Worker {
    int device = 0;
    hdfs3_crc_ctx *ctx = nullptr;
    unsigned long long *d_res = nullptr, *h_res = nullptr;
    size_t res_cap = 0;

    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<int()> job;
    bool has_job = false, done = false, quit = false;
    int rc = 0;
    std::string err;

    void run() {
        (void)hipSetDevice(device);
        hdfs3crc::bind_thread_to_device(device);  // its staging and copies on the GPU's own node
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return has_job || quit; });
            if (quit) return;
            std::function<int()> j = std::move(job);
            has_job = false;
            lk.unlock();
            const int r = j();
            const std::string e = r ? hdfs3_crc_last_error() : std::string();  // thread-local in this thread
            lk.lock();
            rc = r;
            err = e;
            done = true;
            cv.notify_all();
        }
    }
    void post(std::function<int()> j) {
        std::lock_guard<std::mutex> lk(mu);
        job = std::move(j);
        has_job = true;
        done = false;
        cv.notify_all();
    }
    int wait(std::string *msg) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done; });
        if (rc && msg) *msg = err;
        return rc;
    }
    // per-block result words for n blocks (called on the worker thread)
    int reserve(size_t n) {
        if (n <= res_cap) return 0;
        if (d_res) (void)hipFree(d_res);
        if (h_res) (void)hipHostFree(h_res);
        d_res = h_res = nullptr;
        res_cap = 0;
        if (hipMalloc(reinterpret_cast<void **>(&d_res), n * 8) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&h_res), n * 8, hdfs3crc::pinned_host_flags()) != hipSuccess)
            return fail(-ENOMEM, "device %d: result array for %zu blocks", device, n);
        res_cap = n;
        return 0;
    }
};

int device_of(const void *p, int *dev) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return -EINVAL;
    }
    if (a.type != hipMemoryTypeDevice) return -EINVAL;
    *dev = a.device;
    return 0;
}

}  // namespace

struct hdfs3_multi {
    std::vector<Worker *> w;
};

namespace {

// Runs body(worker, block indices of that worker) on every worker that has blocks.
int fan_out(hdfs3_multi *m, size_t n, const std::function<int(Worker &, const std::vector<size_t> &)> &body) {
    const size_t G = m->w.size();
    std::vector<std::vector<size_t>> mine(G);
    for (size_t b = 0; b < n; ++b) mine[b % G].push_back(b);
    for (size_t g = 0; g < G; ++g)
        if (!mine[g].empty()) {
            Worker *wk = m->w[g];
            const std::vector<size_t> *idx = &mine[g];
            wk->post([wk, idx, &body] { return body(*wk, *idx); });
        }
    int rc = 0;
    std::string msg;
    for (size_t g = 0; g < G; ++g)
        if (!mine[g].empty()) {
            std::string e;
            const int r = m->w[g]->wait(&e);
            if (r && !rc) {
                rc = r;
                msg = "device " + std::to_string(m->w[g]->device) + ": " + e;
            }
        }
    if (rc) return fail(rc, "%s", msg.c_str());
    return 0;
}

int check_dev_blocks(hdfs3_multi *m, const hdfs3_dev_block *blocks, size_t n) {
    const size_t G = m->w.size();
    for (size_t b = 0; b < n; ++b) {
        if (!blocks[b].len) continue;
        if (!blocks[b].data || !blocks[b].crc_be) return fail(-EINVAL, "block %zu: null buffer", b);
        int dd = -1, dc = -1;
        const int want = m->w[b % G]->device;
        if (device_of(blocks[b].data, &dd) || device_of(blocks[b].crc_be, &dc) || dd != want || dc != want)
            return fail(-EINVAL, "block %zu must be device memory of device %d (block b -> devices[b %% %zu])", b, want,
                        G);
    }
    return 0;
}

}  // namespace

extern "C" {

int hdfs3_multi_create(const int *devices, int n_devices, hdfs3_multi **out) {
    if (!out || !devices || n_devices <= 0) return fail(-EINVAL, "invalid argument");
    *out = nullptr;
    hdfs3_multi *m = new (std::nothrow) hdfs3_multi();
    if (!m) return fail(-ENOMEM, "hdfs3_multi allocation");
    for (int i = 0; i < n_devices; ++i) {
        Worker *wk = new (std::nothrow) Worker();
        if (!wk) {
            hdfs3_multi_destroy(m);
            return fail(-ENOMEM, "worker allocation");
        }
        wk->device = devices[i];
        m->w.push_back(wk);
        if (int rc = hdfs3_crc_ctx_create(devices[i], &wk->ctx)) {
            hdfs3_multi_destroy(m);
            return rc;
        }
        try {
            wk->th = std::thread([wk] { wk->run(); });
        } catch (const std::system_error &) {  // never across the extern "C" boundary
            hdfs3_multi_destroy(m);
            return fail(-EAGAIN, "worker thread for device %d could not be started", devices[i]);
        }
    }
    *out = m;
    return 0;
}

void hdfs3_multi_destroy(hdfs3_multi *m) {
    if (!m) return;
    for (Worker *wk : m->w) {
        if (wk->th.joinable()) {
            {
                std::lock_guard<std::mutex> lk(wk->mu);
                wk->quit = true;
                wk->cv.notify_all();
            }
            wk->th.join();
        }
        if (wk->ctx) {
            hdfs3crc::DeviceGuard guard(wk->device);  // the caller's current device is left as it was
            hdfs3_crc_ctx_destroy(wk->ctx);
            if (wk->d_res) (void)hipFree(wk->d_res);
            if (wk->h_res) (void)hipHostFree(wk->h_res);
        }
        delete wk;
    }
    delete m;
}

int hdfs3_multi_device_count(hdfs3_multi *m) { return m ? int(m->w.size()) : -EINVAL; }

int hdfs3_crc32c_verify_blocks_multi(hdfs3_multi *m, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc,
                                     int check_short_tail, int64_t *first_bad) {
    if (!m || (n && (!blocks || !first_bad))) return fail(-EINVAL, "invalid argument");
    if (bpc == 0) return fail(-EINVAL, "bytes per checksum must be positive");
    if (int rc = check_dev_blocks(m, blocks, n)) return rc;
    return fan_out(m, n, [&](Worker &wk, const std::vector<size_t> &idx) -> int {
        if (int rc = wk.reserve(idx.size())) return rc;
        hipStream_t s = static_cast<hipStream_t>(hdfs3_crc_ctx_get_stream(wk.ctx));
        if (hipMemsetAsync(wk.d_res, 0, idx.size() * 8, s) != hipSuccess)
            return fail(-EIO, "device %d: result memset failed", wk.device);
        bool prev_verify = false;  // the first launch stays barriered behind the memset
        for (size_t i = 0; i < idx.size(); ++i) {
            const hdfs3_dev_block &b = blocks[idx[i]];
            if (!b.len) continue;
            // every block and word array was resident before the first launch and each verify
            // only reads them: later launches may overlap their predecessor (hdfs3_crc.h)
            if (int rc = hdfs3_crc32c_verify_dev_async_ex(wk.ctx, b.data, b.len, bpc, b.crc_be, check_short_tail,
                                                          reinterpret_cast<uint64_t *>(wk.d_res + i),
                                                          prev_verify ? HDFS3_LAUNCH_OVERLAP_PREVIOUS : 0u))
                return rc;
            prev_verify = true;
        }
        if (hipMemcpyAsync(wk.h_res, wk.d_res, idx.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return fail(-EIO, "device %d: verify failed", wk.device);
        for (size_t i = 0; i < idx.size(); ++i) first_bad[idx[i]] = hdfs3_crc_decode_result(wk.h_res[i]);
        return 0;
    });
}

int hdfs3_crc32c_compute_blocks_multi(hdfs3_multi *m, const hdfs3_dev_block *blocks, size_t n, uint32_t bpc) {
    if (!m || (n && !blocks)) return fail(-EINVAL, "invalid argument");
    if (bpc == 0) return fail(-EINVAL, "bytes per checksum must be positive");
    if (int rc = check_dev_blocks(m, blocks, n)) return rc;
    return fan_out(m, n, [&](Worker &wk, const std::vector<size_t> &idx) -> int {
        for (size_t i : idx)
            if (blocks[i].len)
                if (int rc = hdfs3_crc32c_compute_dev(wk.ctx, blocks[i].data, blocks[i].len, bpc, blocks[i].crc_be))
                    return rc;
        return hdfs3_crc_ctx_synchronize(wk.ctx);
    });
}

int hdfs3_crc32c_verify_host_multi(hdfs3_multi *m, const hdfs3_host_block *blocks, size_t n, uint32_t bpc,
                                   int check_short_tail, int64_t *first_bad) {
    if (!m || (n && (!blocks || !first_bad))) return fail(-EINVAL, "invalid argument");
    return fan_out(m, n, [&](Worker &wk, const std::vector<size_t> &idx) -> int {
        for (size_t i : idx)
            if (int rc = hdfs3_crc32c_verify(wk.ctx, blocks[i].data, blocks[i].len, bpc, blocks[i].crc_be,
                                             check_short_tail, &first_bad[i]))
                return rc;
        return 0;
    });
}

int hdfs3_crc32c_compute_host_multi(hdfs3_multi *m, const hdfs3_host_block *blocks, size_t n, uint32_t bpc) {
    if (!m || (n && !blocks)) return fail(-EINVAL, "invalid argument");
    return fan_out(m, n, [&](Worker &wk, const std::vector<size_t> &idx) -> int {
        for (size_t i : idx)
            if (int rc = hdfs3_crc32c_compute(wk.ctx, blocks[i].data, blocks[i].len, bpc,
                                              const_cast<void *>(blocks[i].crc_be)))
                return rc;
        return 0;
    });
}

}  // extern "C"
