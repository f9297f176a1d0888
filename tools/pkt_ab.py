#!/usr/bin/env python3
"""In-process interleaved A/B of the packet-stream verify (hdfs3_crc32c_verify_packet_stream_dev_async)
against contiguous-block verify of the same payload: 1 GiB of 64 KiB packets in the block reader's
device layout ([128 BE words][64 KiB data] at a 66,048-byte pitch), 2,048 packets (128 MiB of payload)
per launch rotating over 8 streams, the bench's `packets` block shape. Variants via hdfs3x_set_variant
(lab library); each sample = R back-to-back launches, HIP events on the launch stream; N rounds;
median and min per case. Every launch's result slot is checked at the end.

    python tools/pkt_ab.py --variants 0,124 --rounds 7 [--overlap] [--pitch 66048]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--overlap", action="store_true")
    ap.add_argument("--pitch", type=int, default=512 + 65536, help="packet pitch; words at the start, data 512 B in"
                    " (or at pitch - 65536 when the pitch leaves more room)")
    ap.add_argument("--npk", type=int, default=2048, help="packets per launch")
    ap.add_argument("--warm", type=int, default=2000)
    ap.add_argument("--mode", default="verify", choices=["verify", "compute"])
    ap.add_argument("--product", action="store_true", help="the product library (variant 0 only)")
    ap.add_argument("--warm-each", type=int, default=20, help="launches before each timed sample")
    ap.add_argument("--settle", action="store_true", help="settle (poll, then sync) before each timed sample")
    args = ap.parse_args()

    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lib() if args.product else _native.lab()
    if args.product:
        lib.hdfs3x_set_variant = lambda v: None
    dev = torch.device("cuda", 0)
    ctx = CrcContext(0, lib=lib)
    stream = torch.cuda.Stream(device=dev)
    ctx.set_stream(stream.cuda_stream)
    torch.cuda.set_stream(stream)
    bpc, plen, npk, pitch = 512, 65536, args.npk, args.pitch
    nstreams = 8
    data_off = pitch - plen
    crc_off = data_off - 512
    arena = torch.randint(0, 256, (nstreams * npk, pitch), dtype=torch.uint8, device=dev)
    block = torch.empty((nstreams, npk * plen), dtype=torch.uint8, device=dev)
    block.view(-1, plen)[:] = arena[:, data_off:]
    words = torch.empty((nstreams, npk * 512), dtype=torch.uint8, device=dev)
    span = npk * pitch
    ps = ctx.packet_stream(crc_off, data_off, pitch, npk, plen)
    lib.hdfs3x_set_variant(0)
    for s in range(nstreams):
        ctx.compute_dev(block[s].data_ptr(), npk * plen, bpc, words[s].data_ptr())
    torch.cuda.synchronize()
    arena[:, crc_off:crc_off + 512] = words.view(-1, 512)
    scratch = torch.empty_like(words)
    res = torch.zeros(4096, dtype=torch.int64, device=dev)
    base, rp = arena.data_ptr(), res.data_ptr()
    torch.cuda.synchronize()

    def pk(v, i):
        lib.hdfs3x_set_variant(v)
        if args.mode == "verify":
            ctx.verify_packet_stream_async(base + (i % nstreams) * span, span, ps, bpc, rp + 8 * (i % 4096),
                                           overlap_previous=args.overlap and i > 0)
        else:
            ctx.compute_packet_stream_async(base + (i % nstreams) * span, span, ps, bpc)

    def blk(i):
        lib.hdfs3x_set_variant(0)
        if args.mode == "verify":
            ctx.verify_dev_async(block[i % nstreams].data_ptr(), npk * plen, bpc, words[i % nstreams].data_ptr(),
                                 rp + 8 * (i % 4096), overlap_previous=args.overlap and i > 0)
        else:
            ctx.compute_dev(block[i % nstreams].data_ptr(), npk * plen, bpc, scratch[i % nstreams].data_ptr(),
                            overlap_previous=args.overlap and i > 0)

    cases = [(f"packets_v{v}", (lambda v: lambda i: pk(v, i))(v)) for v in
             [int(x) for x in args.variants.split(",")]] + [("contiguous", blk)]
    for i in range(args.warm):
        blk(i)
    torch.cuda.synchronize()
    samples = {n: [] for n, _ in cases}
    for _ in range(args.rounds):
        for name, fn in cases:
            for i in range(args.warm_each):
                fn(i)
            if args.settle:
                done = torch.cuda.Event()
                done.record(stream)
                while not done.query():
                    pass
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(args.reps):
                fn(i)
            e1.record(stream)
            torch.cuda.synchronize()
            samples[name].append(e0.elapsed_time(e1) * 1e3 / args.reps)
    lib.hdfs3x_set_variant(0)
    ok = not bool((res != 0).any().item())
    if args.mode == "compute":  # the packets' words were rewritten in place: they must still verify
        res.zero_()
        ctx.verify_packet_stream_async(base, arena.numel(), ctx.packet_stream(crc_off, data_off, pitch,
                                                                              nstreams * npk, plen), bpc, rp)
        torch.cuda.synchronize()
        ok = ok and int(res[0].item()) == 0
    cmed = statistics.median(samples["contiguous"])
    for name, xs in samples.items():
        med = statistics.median(xs)
        print(json.dumps({"case": name, "mode": args.mode, "overlap": args.overlap, "pitch": pitch,
                          "us_med": round(med, 2), "us_min": round(min(xs), 2),
                          "vs_contiguous": round(cmed / med, 4), "results_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
