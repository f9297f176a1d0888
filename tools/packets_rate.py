#!/usr/bin/env python3
"""Device-resident packet-stream verify/compute rate: a 1 GiB arena of 64 KiB packets in the wire
layout [CRCs][data] (data 16 B aligned), against the contiguous block rate on the same payload.

Lines (GiB/s of payload):
  * sync descriptor API (hdfs3_crc32c_{verify,compute}_packets_dev): host pass + launch + sync
    per call, for variant 0 (constant pitch -> the wave kernel's pitch mode), 53 (the segmented
    kernel's strided launch, the previous production path), 52 (segmented kernel with a
    descriptor array) and 17 (chunk-per-lane packet kernel);
  * async descriptor API (hdfs3_crc32c_*_packets_dev_async): one host pass, no sync, timed
    back to back with HIP events;
  * async stream API (hdfs3_crc32c_*_packet_stream_dev_async): O(1) host work, barriered and
    overlapped (HDFS3_LAUNCH_OVERLAP_PREVIOUS);
  * the contiguous reference: hdfs3_crc32c_verify_dev_async over one 1 GiB block (the same
    payload bytes), barriered and overlapped, and compute_dev.
Verdict target: packet streams within 5 % of the contiguous block rate."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    ctx = CrcContext(0, lib=lib)
    bpc, pkt = 512, 65536
    n = (1 << 30) // pkt
    stride = 512 + pkt  # [128 CRC words][64 KiB data]: data stays 16 B aligned
    arena = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device="cuda")
    block = torch.randint(0, 256, (n * pkt,), dtype=torch.uint8, device="cuda")
    bwords = torch.zeros(n * pkt // bpc * 4, dtype=torch.uint8, device="cuda")
    desc = (_native.PktDesc * n)()
    for i in range(n):
        desc[i].data_off, desc[i].crc_off, desc[i].data_len, desc[i].reserved = i * stride + 512, i * stride, pkt, 0
    ps = CrcContext.packet_stream(0, 512, stride, n, pkt)
    res = torch.zeros(1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.Stream()  # a real stream: the default one's handle is 0, which set_stream reads as "own"
    ctx.set_stream(stream.cuda_stream)
    GiB = n * pkt / 2**30
    bp, bc = ctypes.c_int64(), ctypes.c_int64()
    torch.cuda.synchronize()
    _native.check("compute", lib.hdfs3_crc32c_compute_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n,
                                                                  bpc))
    _native.check("compute", lib.hdfs3_crc32c_compute_dev(ctx.ctx, block.data_ptr(), block.numel(), bpc,
                                                          bwords.data_ptr()))
    torch.cuda.synchronize()

    def timed(fn, reps=30, warm=30):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        host = (time.perf_counter() - t0) / reps
        return e0.elapsed_time(e1) * 1e-3 / reps, host

    out = []
    # ramp the clocks
    for _ in range(300):
        lib.hdfs3_crc32c_verify_dev_async(ctx.ctx, block.data_ptr(), block.numel(), bpc, bwords.data_ptr(), 0,
                                          res.data_ptr())
    torch.cuda.synchronize()
    for rnd in range(2):
        for v in (0, 53, 52, 17):
            lib.hdfs3x_set_variant(v)
            assert lib.hdfs3_crc32c_verify_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n, bpc, 0,
                                                       ctypes.byref(bp), ctypes.byref(bc)) == 0 and bp.value == -1
            tv = timed(lambda: lib.hdfs3_crc32c_verify_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n,
                                                                   bpc, 0, ctypes.byref(bp), ctypes.byref(bc)), 10, 3)
            tc = timed(lambda: lib.hdfs3_crc32c_compute_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n,
                                                                    bpc), 10, 3)
            out.append({"bench": "packets_dev", "api": "sync descriptors", "variant": v, "round": rnd,
                        "verify_GiBps": round(GiB / tv[1], 1), "compute_GiBps": round(GiB / tc[1], 1)})
        lib.hdfs3x_set_variant(0)
        tv = timed(lambda: lib.hdfs3_crc32c_verify_packets_dev_async(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n,
                                                                     bpc, 0, res.data_ptr()))
        tc = timed(lambda: lib.hdfs3_crc32c_compute_packets_dev_async(ctx.ctx, arena.data_ptr(), arena.numel(), desc,
                                                                      n, bpc))
        out.append({"bench": "packets_dev", "api": "async descriptors", "round": rnd,
                    "verify_GiBps": round(GiB / tv[0], 1), "compute_GiBps": round(GiB / tc[0], 1),
                    "verify_us": round(tv[0] * 1e6, 1), "host_us_per_call": round(tv[1] * 1e6, 1)})
        for ovl in (0, 1):
            tv = timed(lambda: lib.hdfs3_crc32c_verify_packet_stream_dev_async(ctx.ctx, arena.data_ptr(), arena.numel(),
                                                                               ctypes.byref(ps), bpc, 0, res.data_ptr(),
                                                                               ovl))
            tb = timed(lambda: lib.hdfs3_crc32c_verify_dev_async_ex(ctx.ctx, block.data_ptr(), block.numel(), bpc,
                                                                    bwords.data_ptr(), 0, res.data_ptr(), ovl))
            out.append({"bench": "packets_dev", "api": "async stream", "overlap": ovl, "round": rnd,
                        "verify_GiBps": round(GiB / tv[0], 1), "verify_us": round(tv[0] * 1e6, 1),
                        "contiguous_block_verify_GiBps": round(GiB / tb[0], 1),
                        "contiguous_block_verify_us": round(tb[0] * 1e6, 1),
                        "ratio_to_contiguous": round(tb[0] / tv[0], 4)})
        tc = timed(lambda: lib.hdfs3_crc32c_compute_packet_stream_dev_async(ctx.ctx, arena.data_ptr(), arena.numel(),
                                                                            ctypes.byref(ps), bpc))
        tb = timed(lambda: lib.hdfs3_crc32c_compute_dev(ctx.ctx, block.data_ptr(), block.numel(), bpc,
                                                        bwords.data_ptr()))
        out.append({"bench": "packets_dev", "api": "async stream compute", "round": rnd,
                    "compute_GiBps": round(GiB / tc[0], 1), "contiguous_block_compute_GiBps": round(GiB / tb[0], 1),
                    "ratio_to_contiguous": round(tb[0] / tc[0], 4)})
    # layout probe: the same stream with every packet's data on a 4 KiB boundary (pitch 68 KiB,
    # words in the 512 B before the data) vs the wire-dense pitch above (64.5 KiB: rounds
    # straddle 4 KiB pages)
    apitch = pkt + 4096
    arena2 = torch.randint(0, 256, (n * apitch,), dtype=torch.uint8, device="cuda")
    ps2 = CrcContext.packet_stream(4096 - 512, 4096, apitch, n, pkt)
    torch.cuda.synchronize()
    lib.hdfs3_crc32c_compute_packet_stream_dev_async(ctx.ctx, arena2.data_ptr(), arena2.numel(), ctypes.byref(ps2), bpc)
    for rnd in range(2):
        for ovl in (0, 1):
            tv = timed(lambda: lib.hdfs3_crc32c_verify_packet_stream_dev_async(ctx.ctx, arena.data_ptr(), arena.numel(),
                                                                               ctypes.byref(ps), bpc, 0, res.data_ptr(),
                                                                               ovl))
            ta = timed(lambda: lib.hdfs3_crc32c_verify_packet_stream_dev_async(
                ctx.ctx, arena2.data_ptr(), arena2.numel(), ctypes.byref(ps2), bpc, 0, res.data_ptr(), ovl))
            tb = timed(lambda: lib.hdfs3_crc32c_verify_dev_async_ex(ctx.ctx, block.data_ptr(), block.numel(), bpc,
                                                                    bwords.data_ptr(), 0, res.data_ptr(), ovl))
            out.append({"bench": "packets_dev", "api": "async stream layout probe", "overlap": ovl, "round": rnd,
                        "pitch_66048_us": round(tv[0] * 1e6, 1), "pitch_69632_aligned_us": round(ta[0] * 1e6, 1),
                        "contiguous_us": round(tb[0] * 1e6, 1)})
    res.zero_()
    torch.cuda.synchronize()
    assert lib.hdfs3_crc32c_verify_packet_stream_dev_async(ctx.ctx, arena.data_ptr(), arena.numel(), ctypes.byref(ps),
                                                           bpc, 0, res.data_ptr(), 0) == 0
    torch.cuda.synchronize()
    assert int(res.item()) == 0, "computed words failed to verify"
    ctx.set_stream(None)
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
