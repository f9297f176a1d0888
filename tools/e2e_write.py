#!/usr/bin/env python3
"""Write path, PCIe-inclusive (docs/DESIGN_HISTORY.md §5.1): hdfsWrite (hdfs3_output_write) of a 1 GiB
host buffer in 1 MiB writes, 128 MiB blocks, 512 B chunks — user bytes copied into pinned
packet arenas, H2D, GPU compute of every chunk's CRC, D2H of the words, packets assembled
and handed to a C sink that reads every packet byte (a stand-in for the pipeline socket).
Batch sizes are swept; the model check (tests/test_output_stream.py) covers correctness.
Reports GiB/s of user data. Never bench `value`."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import OutputStream

    lb = _native.loopback()
    sink = ctypes.cast(lb.hdfs3_loopback_count_sink, ctypes.c_void_p).value
    total = 1 << 30
    data = np.random.default_rng(1).integers(0, 256, size=total, dtype=np.uint8)
    for batch in (16, 64, 256):
        best = 0.0
        for rep in range(3):
            counts = (ctypes.c_uint64 * 3)()
            with OutputStream(block_size=128 << 20, batch_packets=batch, raw_sink=sink,
                              raw_user=ctypes.addressof(counts)) as s:
                t0 = time.perf_counter()
                for off in range(0, total, 1 << 20):
                    s.write(data[off:off + (1 << 20)])
                s.close()
                dt = time.perf_counter() - t0
            best = max(best, total / dt / 2**30)
            # every block: ceil(chunks / 127) data packets + its empty last packet
            blocks, per_block = total // (128 << 20), (128 << 20) // 512
            assert counts[0] == blocks * (-(-per_block // 127) + 1), counts[0]
        print(json.dumps({"bench": "e2e_write", "mode": "hdfsWrite", "bytes": total, "bpc": 512,
                          "batch_packets": batch, "packets": int(counts[0]), "wire_bytes": int(counts[1]),
                          "gib_s": round(best, 2)}), flush=True)
    pipeline_rate(data)


def pipeline_rate(data):
    """hdfsWrite through datanodes (config 5's write twin): OP_WRITE_BLOCK pipelines of 1 and 3
    loopback nodes over 127.0.0.1 TCP; every packet acked by every node, the last node
    verifying every CRC word on its CPU. Socket-inclusive; GPU compute-on-write."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
    from loopback import LoopbackDatanode

    from libhdfs3_amd.engine import OutputStream, Pipeline

    total, bs = data.size, 128 << 20
    for n_nodes in (1, 3):
        nodes = [LoopbackDatanode() for _ in range(n_nodes)]
        for d in nodes:  # verify + ack every packet, skip the in-memory copy (its page faults)
            d.set_store_written(False)
        best = 0.0
        for rep in range(2):
            chain = [("127.0.0.1", d.port) for d in nodes]
            blocks = [(7000 + 100 * rep + i, chain) for i in range(total // bs)]
            with Pipeline(blocks) as pipe:
                t0 = time.perf_counter()
                with OutputStream(block_size=bs, batch_packets=64, pipeline=pipe) as s:
                    for off in range(0, total, 1 << 20):
                        s.write(data[off:off + (1 << 20)])
                dt = time.perf_counter() - t0
                acked = pipe.stats()["block_bytes_acked"]
            assert acked == [bs] * len(blocks), acked
            assert all(d.write_stats()["finalized"] == 0 for d in nodes)
            best = max(best, total / dt / 2**30)
        errs = sum(d.write_stats()["checksum_errors"] for d in nodes)
        for d in nodes:
            d.stop()
        assert errs == 0
        print(json.dumps({"bench": "e2e_write", "mode": "hdfsWrite->pipeline", "nodes": n_nodes, "bytes": total,
                          "bpc": 512, "batch_packets": 64, "gib_s": round(best, 2),
                          "note": "loopback datanodes in this process; the last node verifies every word on its CPU "
                                  "(SSE4.2); nodes do not keep the bytes (store off)"}),
              flush=True)


if __name__ == "__main__":
    main()
