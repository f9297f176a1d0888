#!/usr/bin/env python3
"""Per-open cost of the client drop-ins (docs/DESIGN_HISTORY.md §5.1): libhdfs3 opens one input stream
per file (hdfsOpenFile) and one block reader per block, so small-file reads pay that cost
every time. Times (ms, mean of N):
  ctx          hdfs3_crc_ctx_create + destroy (public API, never pooled)
  input_1mib   hdfs3_input_open + read of a 1 MiB block from the loopback datanode + close
               (the stream's ctx and arenas come from the process-wide pool after the first)
  local_1mib   hdfs3_local_reader open + read of a 1 MiB block file + .meta + close
Prints one JSON line per case."""
import json
import os
import struct
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))  # loopback helper


def main(n=20):
    from libhdfs3_amd.engine import CrcContext, InputStream, LocalBlockReader
    from loopback import LoopbackDatanode

    ctx = CrcContext(0)
    data = np.random.default_rng(1).integers(0, 256, 1 << 20, dtype=np.uint8)
    crc = ctx.compute(data, 512)  # words from the GPU engine (parity is the test suite's job)
    ctx.close()

    def mean_ms(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        return round((time.perf_counter() - t0) / n * 1e3, 3)

    print(json.dumps({"bench": "open_cost", "case": "ctx_create_destroy", "ms": mean_ms(lambda: CrcContext(0).close())}),
          flush=True)
    dn = LoopbackDatanode()
    dn.add_block(1, data, crc, 512)

    def remote():
        with InputStream([(1, data.nbytes, [("127.0.0.1", dn.port)])]) as s:
            assert np.array_equal(s.read_fully(data.nbytes), data)

    print(json.dumps({"bench": "open_cost", "case": "input_open_read_1MiB_close", "ms": mean_ms(remote)}), flush=True)
    dn.stop()
    tmp = tempfile.mkdtemp(prefix="hdfs3_open_")
    d, m = os.path.join(tmp, "blk"), os.path.join(tmp, "blk.meta")
    with open(d, "wb") as f:
        f.write(data.tobytes())
    with open(m, "wb") as f:
        f.write(struct.pack(">hBI", 1, 2, 512) + crc.tobytes())

    def local():
        with LocalBlockReader(d, m) as r:
            assert np.array_equal(r.read_all(data.nbytes), data)

    print(json.dumps({"bench": "open_cost", "case": "local_open_read_1MiB_close", "ms": mean_ms(local)}), flush=True)
    os.remove(d)
    os.remove(m)
    os.rmdir(tmp)


if __name__ == "__main__":
    main()
