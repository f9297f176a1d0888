/*
 * GpuCrc32c — libhdfs3's streaming Checksum interface (src/common/Checksum.h:43-67) over
 * this library's CRC32C engine, for the places that stay streaming: the partial chunk a
 * writer carries across append() calls (OutputStreamImpl.cpp:298-346) and any caller that
 * expects a Checksum object. Batches of whole chunks go to the GPU through the batch calls
 * of hdfs3_crc.h instead.
 *
 * Drop-in for the engine choice at OutputStreamImpl.cpp:55-66, RemoteBlockReader.cpp:
 * 169-184 and LocalBlockReader.cpp:86-98:
 *     checksum = shared_ptr<Checksum>(new GpuCrc32c());
 * Semantics are SWCrc32c/HWCrc32c's: reset() sets the raw state to 0xFFFFFFFF, update()
 * folds bytes in, getValue() returns ~state (0 right after construction or reset()).
 *
 * Header-only; compiled against the reference's own Checksum.h by
 * tests/test_reference_headers.py, which runs the reference KATs (TestChecksum.cpp:83-140)
 * through it. Link with -lhdfs3_crc.
 */
#ifndef HDFS3_INTEGRATION_GPUCRC32C_H
#define HDFS3_INTEGRATION_GPUCRC32C_H

#include "Checksum.h"  /* src/common/Checksum.h of libhdfs3 */
#include "hdfs3_crc.h"

namespace Hdfs {
namespace Internal {

class GpuCrc32c : public Checksum {
public:
    GpuCrc32c() { reset(); }

    uint32_t getValue() override { return ~state; }

    void reset() override { state = 0xFFFFFFFFu; }

    void update(const void *b, int len) override {
        if (len > 0) state = hdfs3_crc32c_update_host(state, b, static_cast<size_t>(len));
    }

    ~GpuCrc32c() override {}

private:
    uint32_t state = 0xFFFFFFFFu;
};

}  // namespace Internal
}  // namespace Hdfs

#endif /* HDFS3_INTEGRATION_GPUCRC32C_H */
