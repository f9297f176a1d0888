"""Config 5 (BASELINE.json): end-to-end, PCIe-inclusive rates of the read path.

  host_verify   hdfs3_crc32c_verify on a 1 GiB host buffer (pinned ring -> H2D -> verify)
  hdfsRead      1 GiB file = 8 x 128 MiB blocks served by the loopback datanode over TCP
                127.0.0.1, read through hdfs3_input_read (InputStreamImpl block walk ->
                hdfs3_block_reader: socket -> pinned arena -> H2D -> packet-kernel verify ->
                caller buffer), verify on vs off
  parallel      8 concurrent streams, one hdfsPread of one whole block each
  readahead     hdfsRead on one stream with block read-ahead (hdfs3_input_set_readahead D)
  local         short-circuit read (hdfs3_local_reader, LocalBlockReader): 8 block files of
                128 MiB + .meta in a temp dir (page-cache resident after writing), 4 MiB reads,
                verify on vs off; 1 stream, and 8 concurrent readers (one block each)

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
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))  # loopback helper

GIB = 1 << 30


def host_verify(ctx, data, crc, bpc, reps):
    bad = ctx.verify(data, bpc, crc)
    assert bad == -1, bad
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.verify(data, bpc, crc)
    dt = (time.perf_counter() - t0) / reps
    return data.nbytes / dt / GIB


def pread_block(blocks, port, i, bsz, out, verify, batch, errors):
    from libhdfs3_amd.engine import InputStream

    try:
        with InputStream([(bid, n, [("127.0.0.1", port)]) for bid, n in blocks], verify=verify,
                         batch_packets=batch) as s:
            got = s.pread_into(i * bsz, out)
            if got != bsz:
                errors.append(f"block {i}: short pread {got}")
    except Exception as e:  # noqa: BLE001 - reported
        errors.append(f"block {i}: {e}")


def diag(dn, blocks, out, data, args):
    """Where a block read spends its time: receive / alloc / launch / wait / deliver (ns)."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import BlockReader

    lib = _native.lab()
    offs = np.cumsum([0] + [n for _, n in blocks])
    for verify in (True, False, True, False):
        acc = np.zeros(5, np.uint64)
        lock = threading.Lock()

        def one(i):
            bid, n = blocks[i]
            with BlockReader("127.0.0.1", dn.port, bid, 0, n, verify=verify, batch_packets=args.batch) as r:
                pos = 0
                while pos < n:
                    got = r.read_into(out, int(offs[i]) + pos, min(args.read_mib << 20, n - pos))
                    assert got > 0
                    pos += got
                t = (ctypes.c_uint64 * 5)()
                _native.check("timing", lib.hdfs3x_block_reader_timing(r.r, t))
                with lock:
                    acc[:] += np.array(list(t), np.uint64)

        t0 = time.perf_counter()
        if args.diag_streams <= 1:  # one block after another on this thread
            for i in range(len(blocks)):
                one(i)
        else:  # every block on its own thread (the parallel_pread shape)
            th = [threading.Thread(target=one, args=(i,)) for i in range(len(blocks))]
            for t in th:
                t.start()
            for t in th:
                t.join()
        off = int(offs[-1])
        dt = time.perf_counter() - t0
        assert np.array_equal(out[:off], data[:off])
        print(json.dumps({"bench": "e2e_diag", "verify": verify, "streams": max(1, args.diag_streams),
                          "gib_s": round(off / dt / GIB, 2), "wall_ms": round(dt * 1e3, 1),
                          **{k: round(float(v) / 1e6, 1) for k, v in
                             zip(["recv_ms", "alloc_ms", "launch_ms", "wait_ms", "deliver_ms"], acc)}}),
              flush=True)


def local_reads(data, crc, args, line):
    """hdfs3_local_reader over block files + .meta (BE16 version 1 | u8 type 2 | BE32 bpc | words)."""
    import shutil
    import struct
    import tempfile

    from libhdfs3_amd.engine import LocalBlockReader

    bsz = args.block_mib << 20
    tmp = tempfile.mkdtemp(prefix="hdfs3_local_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        files = []
        for i in range(args.blocks):
            d, m = os.path.join(tmp, f"blk_{i}"), os.path.join(tmp, f"blk_{i}.meta")
            with open(d, "wb") as f:
                f.write(data[i * bsz:(i + 1) * bsz].tobytes())
            with open(m, "wb") as f:
                f.write(struct.pack(">hBI", 1, 2, args.bpc))
                f.write(crc[4 * (i * bsz // args.bpc): 4 * ((i + 1) * bsz // args.bpc)].tobytes())
            files.append((d, m))
        out = np.empty(args.blocks * bsz, dtype=np.uint8)

        def one(i, verify, errors):
            try:
                with LocalBlockReader(*files[i], verify=verify) as r:
                    pos = 0
                    while pos < bsz:
                        got = r.read_into(out, i * bsz + pos, min(args.read_mib << 20, bsz - pos))
                        if got <= 0:
                            errors.append(f"block {i}: read returned {got} at {pos}")
                            return
                        pos += got
            except Exception as e:  # noqa: BLE001 - reported
                errors.append(f"block {i}: {e}")

        # transport floor: plain buffered reads of the same files into the same buffer
        best = 0.0
        for _ in range(args.reps):
            t0 = time.perf_counter()
            for i, (d, _m) in enumerate(files):
                with open(d, "rb", buffering=0) as f:
                    pos = 0
                    while pos < bsz:
                        n = min(args.read_mib << 20, bsz - pos)
                        got = f.readinto(memoryview(out[i * bsz + pos: i * bsz + pos + n]))
                        assert got and got > 0
                        pos += got
            best = max(best, out.nbytes / (time.perf_counter() - t0) / GIB)
        print(json.dumps({**line, "mode": "plain_file_read", "streams": 1, "read_mib": args.read_mib,
                          "gib_s": round(best, 2), "fs": tmp}), flush=True)
        for verify in (True, False):
            for streams in (1, args.blocks):
                best = 0.0
                rates = []
                cold = []
                for rep in range(args.local_warm + args.reps):
                    errors: list[str] = []
                    t0 = time.perf_counter()
                    if streams == 1:
                        for i in range(args.blocks):
                            one(i, verify, errors)
                    else:
                        th = [threading.Thread(target=one, args=(i, verify, errors)) for i in range(args.blocks)]
                        for t in th:
                            t.start()
                        for t in th:
                            t.join()
                    dt = time.perf_counter() - t0
                    assert not errors, errors
                    if rep < args.local_warm:  # the readers' first resources (pinned windows, contexts)
                        cold.append(round(out.nbytes / dt / GIB, 2))
                        continue
                    best = max(best, out.nbytes / dt / GIB)
                    rates.append(round(out.nbytes / dt / GIB, 2))
                assert np.array_equal(out, data[:out.nbytes])
                out[:] = 0
                staging = {"0": "pread", "1": "mmap"}.get(os.environ.get("HDFS3_LOCAL_MMAP", ""), "default")
                from libhdfs3_amd import _native
                st = _native.PoolStats()
                _native.check("pool_stats", _native.lib().hdfs3_crc_pool_stats_get(ctypes.byref(st)))
                print(json.dumps({**line, "mode": "local_read", "verify": verify, "streams": streams,
                                  "read_mib": args.read_mib, "staging": staging, "gib_s": round(best, 2),
                                  "gib_s_median": sorted(rates)[len(rates) // 2], "gib_s_all": rates, "cold_gib_s": cold,
                                  "pool_retained_pinned_mib": round(st.pinned_bytes / 2**20, 1),
                                  "pool_cap_mib": round(st.pinned_cap_bytes / 2**20, 1)}),
                      flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--block-mib", type=int, default=128)
    ap.add_argument("--bpc", type=int, default=512)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--packet-kib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--local-warm", type=int, default=1,
                    help="short-circuit and read-ahead lines: untimed passes first (reported as cold_gib_s)")
    ap.add_argument("--read-mib", type=int, default=4, help="hdfsRead request size")
    ap.add_argument("--diag", action="store_true", help="per-phase timing of the block reader only")
    ap.add_argument("--diag-streams", type=int, default=1,
                    help="--diag: 1 = blocks one after another, >1 = every block on its own thread")
    ap.add_argument("--local-only", action="store_true", help="only the short-circuit reader lines")
    ap.add_argument("--torch", action="store_true",
                    help="initialise torch's own HIP runtime on cuda:0 first (as bench.py's process has it)")
    ap.add_argument("--only-hdfsread", action="store_true", help="the single-stream hdfsRead lines only")
    ap.add_argument("--no-local", action="store_true", help="skip the short-circuit reader lines")
    ap.add_argument("--reference", action="store_true",
                    help="also the reference's read loop (oracle/_ref HWCrc32c) on the same stream: 1 and 8 threads")
    ap.add_argument("--readahead", default="1,2,3,7",
                    help="block read-ahead depths of the extra single-stream hdfsRead lines ('' = none)")
    args = ap.parse_args()

    if args.torch:
        import torch
        _keep = torch.empty(1 << 30, dtype=torch.uint8, device="cuda:0")  # noqa: F841 (held for the run)
        torch.cuda.synchronize()
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    bsz = args.block_mib << 20
    total = args.blocks * bsz
    ctx = CrcContext(0, lib=_native.lab())
    # a deterministic 1 GiB "file" and its .meta words, computed on the GPU (checked below)
    rng = np.random.default_rng(0x5EED)
    data = rng.integers(0, 256, size=total, dtype=np.uint8)
    crc = ctx.compute(data, args.bpc)
    line = {"bench": "e2e", "bytes": total, "bpc": args.bpc}
    if args.local_only:
        local_reads(data, crc, args, line)
        ctx.close()
        return

    # (the words' parity with the reference is the -m gpu suite's job; this tool only times)
    print(json.dumps({**line, "mode": "host_verify_pageable",
                      "gib_s": round(host_verify(ctx, data, crc, args.bpc, args.reps), 2)}), flush=True)
    lib = _native.lab()
    hp = ctypes.c_void_p()
    _native.check("hdfs3_host_malloc_pinned", lib.hdfs3_host_malloc_pinned(ctypes.byref(hp), total))
    pinned = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(hp.value))
    pinned[:] = data
    print(json.dumps({**line, "mode": "host_verify_pinned",
                      "gib_s": round(host_verify(ctx, pinned, crc, args.bpc, args.reps), 2)}), flush=True)
    del pinned
    lib.hdfs3_host_free_pinned(hp)

    from loopback import LoopbackDatanode
    from libhdfs3_amd.engine import InputStream

    dn = LoopbackDatanode(packet_bytes=args.packet_kib << 10)
    blocks = []
    for i in range(args.blocks):
        d = data[i * bsz:(i + 1) * bsz]
        c = crc[4 * (i * bsz // args.bpc): 4 * ((i + 1) * bsz // args.bpc)]
        dn.add_block(10 + i, d, c, args.bpc)
        blocks.append((10 + i, bsz))
    out = np.empty(total, dtype=np.uint8)
    if args.diag:
        try:
            diag(dn, blocks, out, data, args)
        finally:
            dn.stop()
        return
    try:
        for verify in (True, False):
            for mode in (("hdfsRead",) if args.only_hdfsread else ("hdfsRead", "parallel_pread")):
                best = 0.0
                for _ in range(args.reps):
                    errors: list[str] = []
                    t0 = time.perf_counter()
                    if mode == "hdfsRead":
                        with InputStream([(b, n, [("127.0.0.1", dn.port)]) for b, n in blocks], verify=verify,
                                         batch_packets=args.batch) as s:
                            pos = 0
                            while pos < total:
                                got = s.read_into(out, pos, min(args.read_mib << 20, total - pos))
                                assert got > 0
                                pos += got
                    else:
                        th = [threading.Thread(target=pread_block,
                                               args=(blocks, dn.port, i, bsz, out[i * bsz:(i + 1) * bsz], verify,
                                                     args.batch, errors)) for i in range(args.blocks)]
                        for t in th:
                            t.start()
                        for t in th:
                            t.join()
                    dt = time.perf_counter() - t0
                    assert not errors, errors
                    best = max(best, total / dt / GIB)
                assert np.array_equal(out, data)
                out[:] = 0
                print(json.dumps({**line, "mode": mode, "verify": verify, "streams": 1 if mode == "hdfsRead"
                                  else args.blocks, "batch_packets": args.batch, "packet_kib": args.packet_kib,
                                  "gib_s": round(best, 2)}), flush=True)
        if args.reference:
            from loopback import reference_read_block

            for streams in (1, args.blocks):
                for verify in (True, False):
                    best = 0.0
                    for _ in range(args.reps):
                        errors: list[str] = []

                        def one(i):
                            try:
                                reference_read_block(dn.port, blocks[i][0], bsz, out, i * bsz, verify=verify)
                            except Exception as e:  # noqa: BLE001 - reported
                                errors.append(f"block {i}: {e}")

                        t0 = time.perf_counter()
                        if streams == 1:
                            for i in range(args.blocks):
                                one(i)
                        else:
                            th = [threading.Thread(target=one, args=(i,)) for i in range(args.blocks)]
                            for t in th:
                                t.start()
                            for t in th:
                                t.join()
                        dt = time.perf_counter() - t0
                        assert not errors, errors
                        best = max(best, total / dt / GIB)
                    assert np.array_equal(out, data)
                    out[:] = 0
                    print(json.dumps({**line, "mode": "reference_read_loop", "verify": verify, "streams": streams,
                                      "engine": "oracle/_ref HWCrc32c (RemoteBlockReader loop)",
                                      "gib_s": round(best, 2)}), flush=True)
        # single-stream hdfsRead with block read-ahead (hdfs3_input_set_readahead): blocks
        # i+1 .. i+D read and verified by background threads while block i is consumed
        def pool_mib():
            st = _native.PoolStats()
            _native.check("pool_stats", _native.lib().hdfs3_crc_pool_stats_get(ctypes.byref(st)))
            return round(st.pinned_bytes / 2**20, 1), round(st.pinned_cap_bytes / 2**20, 1)

        for ahead in ([] if args.only_hdfsread else [int(x) for x in args.readahead.split(",") if x]):
            best = 0.0
            rates = []
            cold = []
            for rep in range(args.local_warm + args.reps):
                t0 = time.perf_counter()
                with InputStream([(b, n, [("127.0.0.1", dn.port)]) for b, n in blocks], verify=True,
                                 batch_packets=args.batch) as s:
                    s.set_readahead(ahead)
                    pos = 0
                    while pos < total:
                        got = s.read_into(out, pos, min(args.read_mib << 20, total - pos))
                        assert got > 0
                        pos += got
                dt = time.perf_counter() - t0
                if rep < args.local_warm:  # the stream's first rings (pinned arenas, contexts)
                    cold.append(round(total / dt / GIB, 2))
                    continue
                best = max(best, total / dt / GIB)
                rates.append(round(total / dt / GIB, 2))
            assert np.array_equal(out, data)
            out[:] = 0
            retained, cap = pool_mib()
            print(json.dumps({**line, "mode": "hdfsRead_readahead", "verify": True, "streams": 1,
                              "readahead_blocks": ahead, "batch_packets": args.batch,
                              "packet_kib": args.packet_kib, "gib_s": round(best, 2),
                              "gib_s_median": sorted(rates)[len(rates) // 2], "gib_s_all": rates, "cold_gib_s": cold,
                              "pool_retained_pinned_mib": retained, "pool_cap_mib": cap}), flush=True)
    finally:
        dn.stop()
    if not args.only_hdfsread and not args.no_local:
        local_reads(data, crc, args, line)
    ctx.close()


if __name__ == "__main__":
    main()
