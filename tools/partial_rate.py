#!/usr/bin/env python3
"""Device-resident rates of the round-6 partial-round paths (one JSON line per row):

  * writer_batch: the output stream's 64-packet batch at bpc 512 (127 chunks = 65,024 B per packet,
    slots at a 65,568-byte stride, words compact after them), compute and verify through the
    packets API (descriptors, as output_stream.cpp launches it), barriered, against the reader's
    dense 4 MiB batch verify (one contiguous block);
  * ragged_<bpc>: ~1 GiB descriptor lists of packets at irregular offsets (not one constant-pitch
    stream): 64-127 chunks at bpc 512 (the segmented kernel), 2-5 chunks at bpc 12 KiB / 64 KiB
    (segment piece CRCs + per-segment combine);
  * stream_<bpc>: 1 GiB-class wire streams ([words][data] per packet) whose packets do not hold a
    power-of-two number of whole rounds: 127-chunk packets at bpc 512, and 60 KiB packets of 12 KiB /
    20 KiB chunks (5 / 3 chunks, 15 rounds: the pitch walk's pieces + combine), verify and compute
    (hdfs3_crc32c_*_packet_stream_dev_async), against a contiguous block of the same payload.

Every row's results are checked (clean verifies report nothing, computed words verify)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import argparse

    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="", help="lab variants for the writer-batch row (lab library)")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",") if v]
    lib = _native.lab() if variants else _native.lib()
    ctx = CrcContext(0, lib=lib)
    stream = torch.cuda.Stream()
    ctx.set_stream(stream.cuda_stream)
    torch.cuda.set_stream(stream)
    res = torch.zeros(512, dtype=torch.int64, device="cuda")
    rp = res.data_ptr()

    def timed(fn, n=200, warm=50, reps=5):
        out = []
        for _ in range(reps):
            for i in range(warm):
                fn(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(n):
                fn(i)
            e1.record(stream)
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) * 1e3 / n)
        return sorted(out)[reps // 2]

    # writer batch (bench.py writer_batch_layout, without the pairing)
    bpc, npk, nbat = 512, 64, 16
    cpp = (65536 - 31 + bpc + 3) // (bpc + 4)
    plen = cpp * bpc
    lead = (31 + 4 * cpp + 15) // 16 * 16
    stride = lead + (plen + 15) // 16 * 16
    crc_region = stride * npk
    span = crc_region + 4 * cpp * npk
    span += (-span) % 4096
    arena = torch.randint(0, 256, (nbat, span), dtype=torch.uint8, device="cuda")
    descs = CrcContext._descs([(lead + stride * p, crc_region + 4 * cpp * p, plen) for p in range(npk)])
    ab = arena.data_ptr()
    dense = torch.randint(0, 256, (nbat, 32768 + (4 << 20)), dtype=torch.uint8, device="cuda")
    db = dense.data_ptr()
    for b in range(nbat):
        ctx.compute_packets_dev_async(ab + b * span, span, descs, bpc)
        ctx.compute_dev(db + b * dense.shape[1] + 32768, 4 << 20, bpc, db + b * dense.shape[1])
    torch.cuda.synchronize()
    for rnd in range(2 if variants else 1):
        for v in variants or [0]:
            if variants:
                lib.hdfs3x_set_variant(v)
            tc = timed(lambda i: ctx.compute_packets_dev_async(ab + (i % nbat) * span, span, descs, bpc))
            tv = timed(lambda i: ctx.verify_packets_dev_async(ab + (i % nbat) * span, span, descs, bpc,
                                                              rp + 8 * (i % 512)))
            if variants:  # the reader's contiguous batch under production (the variants are pitch-walk ones)
                lib.hdfs3x_set_variant(0)
            td = timed(lambda i: ctx.verify_dev_async(db + (i % nbat) * dense.shape[1] + 32768, 4 << 20, bpc,
                                                      db + (i % nbat) * dense.shape[1], rp + 8 * (i % 512)))
            torch.cuda.synchronize()
            assert not bool(res.any().item()), "writer batch: clean verify reported a bad chunk"
            alg = npk * cpp * (bpc + 4)
            print(json.dumps({"row": "writer_batch", "variant": v, "round": rnd, "bpc": bpc, "packets": npk,
                              "chunks_per_packet": cpp, "compute_us": round(tc, 2), "verify_us": round(tv, 2),
                              "reader_dense_verify_us": round(td, 2), "compute_GBps": round(alg / tc / 1e3, 1),
                              "compute_vs_reader_dense": round(tc / td, 3)}), flush=True)
    if variants:
        for v in variants:  # every variant's words verify under production
            lib.hdfs3x_set_variant(v)
            arena[:, crc_region:crc_region + 4 * cpp * npk] = 0
            for b in range(nbat):
                ctx.compute_packets_dev_async(ab + b * span, span, descs, bpc)
            lib.hdfs3x_set_variant(0)
            res.zero_()
            for b in range(nbat):
                ctx.verify_packets_dev_async(ab + b * span, span, descs, bpc, rp + 8 * b)
            torch.cuda.synchronize()
            assert not bool(res.any().item()), f"variant {v}: computed words fail to verify"
    del arena, dense

    # ragged descriptor lists (not one constant-pitch stream) at bpc = R x 4096, ~1 GiB: the segmented
    # kernel's piece CRCs + the per-segment combine (round 6); with --variants 0,17 beside the
    # chunk-per-lane packet kernel it replaced (lab 17)
    import numpy as np
    for bpc in (512, 12288, 65536):
        rng = np.random.default_rng(bpc)
        descs_l, off = [], 16
        while off < (1 << 30):
            s = int(rng.integers(2, 6)) * bpc if bpc > 4096 else int(rng.integers(64, 128)) * bpc
            wb = 4 * (s // bpc)
            doff = off + wb
            doff += (-doff) % 16
            descs_l.append((doff, off, s))
            off = doff + s + 16 * int(rng.integers(0, 3))
        arena = torch.randint(0, 256, (off + 64,), dtype=torch.uint8, device="cuda")
        d = CrcContext._descs(descs_l)
        ap_ = arena.data_ptr()
        payload = sum(x[2] for x in descs_l)
        ctx.compute_packets_dev_async(ap_, arena.numel(), d, bpc)
        torch.cuda.synchronize()
        for v in (variants or [0]):
            if variants:
                lib.hdfs3x_set_variant(v)
            res.zero_()
            tv = timed(lambda i: ctx.verify_packets_dev_async(ap_, arena.numel(), d, bpc, rp + 8 * (i % 512)),
                       n=10, warm=3, reps=3)
            tc = timed(lambda i: ctx.compute_packets_dev_async(ap_, arena.numel(), d, bpc), n=10, warm=3, reps=3)
            torch.cuda.synchronize()
            assert not bool(res.any().item()), f"ragged bpc {bpc} variant {v}: clean verify reported a bad chunk"
            print(json.dumps({"row": f"ragged_{bpc}", "variant": v, "bpc": bpc, "packets": len(descs_l),
                              "payload_bytes": payload, "verify_us": round(tv, 1), "compute_us": round(tc, 1),
                              "verify_TiBps": round(payload / tv / 1e-6 / 2**40, 3),
                              "compute_TiBps": round(payload / tc / 1e-6 / 2**40, 3)}), flush=True)
        if variants:
            lib.hdfs3x_set_variant(0)
        del arena

    # wire streams of ~1 GiB payload
    for bpc, cpp in ((512, 127), (12288, 5), (20480, 3)):
        plen = bpc * cpp
        wb = 4 * cpp
        doff = (16 + wb + 15) // 16 * 16
        pitch = (doff + plen + 15) // 16 * 16
        n = (1 << 30) // plen
        a = torch.randint(0, 256, (n * pitch,), dtype=torch.uint8, device="cuda")
        ps = CrcContext.packet_stream(16, doff, pitch, n, plen)
        blk = torch.randint(0, 256, (n * plen,), dtype=torch.uint8, device="cuda")
        bw = torch.zeros(n * wb, dtype=torch.uint8, device="cuda")
        ctx.compute_packet_stream_async(a.data_ptr(), a.numel(), ps, bpc)
        ctx.compute_dev(blk.data_ptr(), blk.numel(), bpc, bw.data_ptr())
        torch.cuda.synchronize()
        res.zero_()
        tv = timed(lambda i: ctx.verify_packet_stream_async(a.data_ptr(), a.numel(), ps, bpc, rp + 8 * (i % 512)),
                   n=20, warm=5, reps=3)
        tc = timed(lambda i: ctx.compute_packet_stream_async(a.data_ptr(), a.numel(), ps, bpc), n=20, warm=5, reps=3)
        tcv = {}
        for v in variants:  # lab variants of the stream compute, interleaved twice, their words checked
            for _ in range(2):
                lib.hdfs3x_set_variant(v)
                tcv.setdefault(v, []).append(
                    timed(lambda i: ctx.compute_packet_stream_async(a.data_ptr(), a.numel(), ps, bpc),
                          n=20, warm=5, reps=3))
                lib.hdfs3x_set_variant(0)
                tcv.setdefault(0, []).append(
                    timed(lambda i: ctx.compute_packet_stream_async(a.data_ptr(), a.numel(), ps, bpc),
                          n=20, warm=5, reps=3))
            lib.hdfs3x_set_variant(v)
            ctx.compute_packet_stream_async(a.data_ptr(), a.numel(), ps, bpc)
            lib.hdfs3x_set_variant(0)
            torch.cuda.synchronize()
            res.zero_()
            ctx.verify_packet_stream_async(a.data_ptr(), a.numel(), ps, bpc, rp)
            torch.cuda.synchronize()
            assert not bool(res.any().item()), f"stream bpc {bpc} variant {v}: computed words fail to verify"
        tb = timed(lambda i: ctx.verify_dev_async(blk.data_ptr(), blk.numel(), bpc, bw.data_ptr(), rp + 8 * (i % 512)),
                   n=20, warm=5, reps=3)
        torch.cuda.synchronize()
        assert not bool(res.any().item()), f"stream bpc {bpc}: clean verify reported a bad chunk"
        payload = n * plen
        print(json.dumps({"row": f"stream_{bpc}", "bpc": bpc, "packets": n, "packet_bytes": plen,
                          "verify_us": round(tv, 1), "compute_us": round(tc, 1), "contiguous_verify_us": round(tb, 1),
                          "verify_TiBps": round(payload / tv / 1e-6 / 2**40, 3),
                          "compute_TiBps": round(payload / tc / 1e-6 / 2**40, 3),
                          "contiguous_verify_TiBps": round(payload / tb / 1e-6 / 2**40, 3),
                          "compute_us_by_variant": {str(k): [round(x, 1) for x in v] for k, v in tcv.items()}}),
              flush=True)
        del a, blk, bw
    ctx.set_stream(None)


if __name__ == "__main__":
    main()
