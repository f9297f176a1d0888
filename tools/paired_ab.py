#!/usr/bin/env python3
"""Paired-region A/B in the bench's own form (bench.py paired_regions): per repetition, one region per
case — 50 warmup launches, settle, n timed launches between HIP events on the launch stream, the first
barriered and the rest overlapped (HDFS3_LAUNCH_OVERLAP_PREVIOUS) unless --barriered — over 128 MiB
blocks rotating through 8 (1 GiB). Cases: mode:variant (lab library), e.g. verify:0 compute:0 compute:118.
Medians over the repetitions; compute results are not checked (diagnostic variants are wrong on purpose).

    python tools/paired_ab.py --cases verify:0,compute:0,compute:118 --reps 5 --n 200
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
    ap.add_argument("--cases", default="verify:0,compute:0")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--bpc", type=int, default=512)
    ap.add_argument("--block-mib", type=int, default=128)
    ap.add_argument("--barriered", action="store_true")
    ap.add_argument("--prepass", type=int, default=2000)
    args = ap.parse_args()
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx = CrcContext(0, lib=lib)
    ctx.set_stream(stream.cuda_stream)
    bb, bpc, nb = args.block_mib << 20, args.bpc, 8
    data = torch.randint(0, 256, (nb, bb), dtype=torch.uint8, device=dev)
    words = torch.empty((nb, bb // bpc * 4), dtype=torch.uint8, device=dev)
    out = torch.empty_like(words)
    for b in range(nb):
        ctx.compute_dev(data[b].data_ptr(), bb, bpc, words[b].data_ptr())
    torch.cuda.synchronize()
    res = torch.zeros(256, dtype=torch.int64, device=dev)
    dp = [data[b].data_ptr() for b in range(nb)]
    wp = [words[b].data_ptr() for b in range(nb)]
    op = [out[b].data_ptr() for b in range(nb)]
    ov = not args.barriered

    def launch(mode, i):
        if mode == "verify":
            ctx.verify_dev_async(dp[i % nb], bb, bpc, wp[i % nb], res.data_ptr() + 8 * (i % 256),
                                 overlap_previous=ov and i > 0)
        else:
            ctx.compute_dev(dp[i % nb], bb, bpc, op[i % nb], overlap_previous=ov and i > 0)

    def settle():
        e = torch.cuda.Event()
        e.record(stream)
        while not e.query():
            pass
        torch.cuda.synchronize()

    cases = [(c.split(":")[0], int(c.split(":")[1])) for c in args.cases.split(",")]
    for i in range(args.prepass):
        launch("verify", i)
    torch.cuda.synchronize()
    times = {c: [] for c in cases}
    for _ in range(args.reps):
        for mode, v in cases:
            lib.hdfs3x_set_variant(v)
            for i in range(50):
                launch(mode, i)
            settle()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(args.n):
                launch(mode, i)
            e1.record(stream)
            torch.cuda.synchronize()
            times[(mode, v)].append(e0.elapsed_time(e1) * 1e3 / args.n)
    lib.hdfs3x_set_variant(0)
    ok = not bool((res != 0).any().item())
    base = statistics.median(times[cases[0]])
    for (mode, v), t in times.items():
        m = statistics.median(t)
        print(json.dumps({"mode": mode, "variant": v, "bpc": bpc, "block_mib": args.block_mib,
                          "overlapped": ov, "us_med": round(m, 3), "us_all": [round(x, 2) for x in t],
                          "vs_first": round(base / m, 4), "verify_results_clean": ok}), flush=True)


if __name__ == "__main__":
    main()
