#!/usr/bin/env python3
"""In-process interleaved A/B of kernel variants (hdfs3x_set_variant), per
cdna_hip_programming.md §5.4 rule 24: N variants x M rounds in ONE process, report
median and min. Each timed sample = R back-to-back launches over 128 MiB blocks
rotating through 8 blocks (1 GiB + CRCs, past the 256 MiB Infinity Cache).

    python tools/ab.py --variants 0,1 --bpc 512,2048,4096 --rounds 7
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
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--bpc", default="512")
    ap.add_argument("--mode", default="verify")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=24)
    ap.add_argument("--ref", action="store_true", help="also time coalesced-read probes")
    ap.add_argument("--streams", default="1", help="comma list: launches alternate over S streams")
    ap.add_argument("--block-mib", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--warm", type=int, default=2000, help="launches of variant 0 before the first sample "
                                                           "(the GPU needs ~25 ms of load to leave its idle clock)")
    ap.add_argument("--overlap", action="store_true",
                    help="launches after the first of each timed batch use HDFS3_LAUNCH_OVERLAP_PREVIOUS")
    args = ap.parse_args()

    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    dev = torch.device("cuda", 0)
    nstreams = [int(x) for x in args.streams.split(",")]
    ctxs = [CrcContext(0, lib=_native.lab()) for _ in range(max(nstreams))]
    streams = [torch.cuda.Stream(device=dev) for _ in ctxs]
    for c, st in zip(ctxs, streams):
        c.set_stream(st.cuda_stream)
    ctx = ctxs[0]
    torch.cuda.set_stream(streams[0])
    blocks, bb = args.blocks, args.block_mib << 20
    data = torch.randint(0, 256, (blocks, bb), dtype=torch.uint8, device=dev)
    sink = torch.zeros(16, dtype=torch.int32, device=dev)
    res = torch.zeros(4096, dtype=torch.int64, device=dev)
    variants = [int(v) for v in args.variants.split(",")]
    out = []
    for bpc in [int(b) for b in args.bpc.split(",")]:
        nch = bb // bpc
        crc = torch.empty((blocks, 4 * nch), dtype=torch.uint8, device=dev)
        lib.hdfs3x_set_variant(0)
        for b in range(blocks):
            ctx.compute_dev(data[b].data_ptr(), bb, bpc, crc[b].data_ptr())
        ref_crc = crc.clone()
        torch.cuda.synchronize()

        def run(v, i, ns):
            lib.hdfs3x_set_variant(v)
            c = ctxs[i % ns]
            if args.mode == "verify":
                c.verify_dev_async(data[i % blocks].data_ptr(), bb, bpc, crc[i % blocks].data_ptr(),
                                   res.data_ptr() + 8 * (i % 4096), overlap_previous=args.overlap and i > 0)
            else:
                c.compute_dev(data[i % blocks].data_ptr(), bb, bpc, crc[i % blocks].data_ptr(),
                              overlap_previous=args.overlap and i > 0)

        cases = [("v%d_s%d" % (v, ns), (lambda v, ns: (lambda i: run(v, i, ns)))(v, ns))
                 for v in variants for ns in nstreams]
        if args.ref:
            cases.append(("coalesced_read_G8", lambda i: lib.hdfs3x_lane_read(
                ctx.ctx, data[i % blocks].data_ptr(), bb, 512 | (2 << 16), sink.data_ptr())))
        samples = {name: [] for name, _ in cases}
        for i in range(args.warm):
            run(0, i, 1)
        for name, fn in cases:  # warm
            for i in range(4):
                fn(i)
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for name, fn in cases:
                # wall time over the whole batch (multi-stream launches overlap)
                torch.cuda.synchronize()
                import time
                t0 = time.perf_counter()
                for i in range(args.reps):
                    fn(i)
                torch.cuda.synchronize()
                samples[name].append((time.perf_counter() - t0) * 1e6 / args.reps)
        bad = bool((res != 0).any().item()) if args.mode == "verify" else False
        same = bool(torch.equal(crc, ref_crc))
        for name, xs in samples.items():
            med = statistics.median(xs)
            out.append({"bpc": bpc, "mode": args.mode, "case": name, "us_med": round(med, 2),
                        "us_min": round(min(xs), 2), "GBps_med": round(bb / med / 1e3, 1),
                        "alg_GBps_med": round(nch * (bpc + 4) / med / 1e3, 1),
                        "results_ok": (not bad) and same})
    lib.hdfs3x_set_variant(0)
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
