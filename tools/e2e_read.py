"""Config 5 (BASELINE.json): end-to-end, PCIe-inclusive rates of the read path.

  host_verify   hdfs3_crc32c_verify on a 1 GiB host buffer (pinned ring -> H2D -> verify)
  loopback      1 GiB file = 8 x 128 MiB blocks served by the loopback datanode over TCP
                127.0.0.1, read through hdfs3_block_reader (socket -> pinned arena -> H2D ->
                packet-kernel verify -> caller buffer), verify on vs off, 1 reader reading the
                blocks in turn (InputStreamImpl order) and 8 concurrent readers (one per block)

The datanode thread and the reader share the host's cores, so the loopback numbers bound
the client from below; the verify-off line is the same transport without the GPU work.
Prints one JSON line per measurement; these are DESIGN.md numbers, never bench `value`.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

GIB = 1 << 30


def host_verify(ctx, data, crc, bpc, reps):
    bad = ctx.verify(data, bpc, crc)
    assert bad == -1, bad
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.verify(data, bpc, crc)
    dt = (time.perf_counter() - t0) / reps
    return data.nbytes / dt / GIB


def read_block(port, bid, nbytes, out, verify, batch, errors):
    from libhdfs3_amd.engine import BlockReader

    try:
        with BlockReader("127.0.0.1", port, bid, 0, nbytes, verify=verify, batch_packets=batch) as r:
            pos = 0
            while pos < nbytes:
                got = r.read_into(out, pos, min(4 << 20, nbytes - pos))
                if got == 0:
                    break
                pos += got
            if pos != nbytes:
                errors.append(f"block {bid}: short read {pos}")
    except Exception as e:  # noqa: BLE001 - reported
        errors.append(f"block {bid}: {e}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--block-mib", type=int, default=128)
    ap.add_argument("--bpc", type=int, default=512)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--packet-kib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    bsz = args.block_mib << 20
    total = args.blocks * bsz
    ctx = CrcContext(0)
    # a deterministic 1 GiB "file" and its .meta words, computed on the GPU (checked below)
    rng = np.random.default_rng(0x5EED)
    data = rng.integers(0, 256, size=total, dtype=np.uint8)
    crc = ctx.compute(data, args.bpc)
    line = {"bench": "e2e", "bytes": total, "bpc": args.bpc}

    # (the words' parity with the reference is the -m gpu suite's job; this tool only times)
    print(json.dumps({**line, "mode": "host_verify_pageable",
                      "gib_s": round(host_verify(ctx, data, crc, args.bpc, args.reps), 2)}), flush=True)
    lib = _native.lib()
    hp = ctypes.c_void_p()
    _native.check("hdfs3_host_malloc_pinned", lib.hdfs3_host_malloc_pinned(ctypes.byref(hp), total))
    pinned = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(hp.value))
    pinned[:] = data
    print(json.dumps({**line, "mode": "host_verify_pinned",
                      "gib_s": round(host_verify(ctx, pinned, crc, args.bpc, args.reps), 2)}), flush=True)
    del pinned
    lib.hdfs3_host_free_pinned(hp)

    lb = _native.loopback()
    port = ctypes.c_int(0)
    assert lb.hdfs3_loopback_start(ctypes.byref(port)) == 0
    lb.hdfs3_loopback_set_packet_bytes(args.packet_kib << 10)
    blocks = []
    for i in range(args.blocks):
        d = data[i * bsz:(i + 1) * bsz]
        c = crc[4 * (i * bsz // args.bpc): 4 * ((i + 1) * bsz // args.bpc)]
        assert lb.hdfs3_loopback_add_block(10 + i, d.ctypes.data, d.nbytes, c.ctypes.data, args.bpc, 2) == 0
        blocks.append((d, c))
    out = np.empty(total, dtype=np.uint8)
    try:
        for verify in (True, False):
            for readers in (1, args.blocks):
                best = 0.0
                for _ in range(args.reps):
                    errors: list[str] = []
                    t0 = time.perf_counter()
                    if readers == 1:
                        for i in range(args.blocks):
                            read_block(port.value, 10 + i, bsz, out[i * bsz:(i + 1) * bsz], verify, args.batch, errors)
                    else:
                        th = [threading.Thread(target=read_block,
                                               args=(port.value, 10 + i, bsz, out[i * bsz:(i + 1) * bsz], verify,
                                                     args.batch, errors)) for i in range(args.blocks)]
                        for t in th:
                            t.start()
                        for t in th:
                            t.join()
                    dt = time.perf_counter() - t0
                    assert not errors, errors
                    best = max(best, total / dt / GIB)
                assert np.array_equal(out, data)
                print(json.dumps({**line, "mode": "loopback_read", "verify": verify, "readers": readers,
                                  "batch_packets": args.batch, "packet_kib": args.packet_kib,
                                  "gib_s": round(best, 2)}), flush=True)
    finally:
        lb.hdfs3_loopback_stop()
    ctx.close()


if __name__ == "__main__":
    main()
