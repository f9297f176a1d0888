#!/usr/bin/env python3
"""Per-launch shader clock and timing of short regions (why the driver's
20-launch form runs slower than the steady state). Every launch of the CRC verify (lab variant 125 =
production + clock stamps) and of the plain stream read records, from workgroup 0, {s_memtime,
s_memrealtime} at its start and end (LabClock, crc32c_device.h): the shader clock during that
workgroup's life is 100 MHz x d(memtime) / d(realtime), and realtime also places every launch's start.

Phases, each a region of K launches of one 128 MiB block each (8 rotating blocks), HIP events around:
  bench     the bench's form: 2000 barriered launches, W warmup, settle (host polls, then sync), K timed
            (first barriered, the rest overlapped)
  steady    the same right after, with max(K, 200) launches
  busy      W warmup, then a GPU-side spin (no idle, no memory traffic) of --spin-us instead of the
            host settle, then K: the GPU never goes idle before the region
  queued    K launches queued behind 500 others with no settle at all
for the CRC verify and for the plain read of the same shape.

    python tools/clock_ramp.py [--k 20] [--w 5] [--reps 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--w", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--spin-us", type=float, default=300.0)
    ap.add_argument("--read-grid", type=int, default=-512)
    ap.add_argument("--kinds", default="crc,read", help="comma list of crc (verify), compute, read")
    ap.add_argument("--phases", default="bench,steady,busy,queued")
    args = ap.parse_args()

    import numpy as np
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    dev = torch.device("cuda", 0)
    ctx = CrcContext(0, lib=lib)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    nb, bb, bpc = 8, 128 << 20, 512
    data = torch.randint(0, 256, (nb, bb), dtype=torch.uint8, device=dev)
    crc = torch.empty((nb, 4 * (bb // bpc)), dtype=torch.uint8, device=dev)
    for b in range(nb):
        ctx.compute_dev(data[b].data_ptr(), bb, bpc, crc[b].data_ptr())
    res = torch.zeros(8192, dtype=torch.int64, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    cap = 1 << 16
    stamps = torch.zeros(cap * 4, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    dp = [data[b].data_ptr() for b in range(nb)]
    cp = [crc[b].data_ptr() for b in range(nb)]
    rp = res.data_ptr()
    # torch.cuda._sleep takes GPU cycles; calibrate against events
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    torch.cuda._sleep(1_000_000)
    e1.record(stream)
    torch.cuda.synchronize()
    cycles_per_us = 1_000_000 / (e0.elapsed_time(e1) * 1e3)

    def crc_launch(i, overlap):
        ctx.verify_dev_async(dp[i % nb], bb, bpc, cp[i % nb], rp + 8 * (i % 8192), overlap_previous=overlap and i > 0)

    scratch = torch.empty_like(crc)
    sp = [scratch[b].data_ptr() for b in range(nb)]

    def compute_launch(i, overlap):
        ctx.compute_dev(dp[i % nb], bb, bpc, sp[i % nb], overlap_previous=overlap and i > 0)

    def read_launch(i, overlap):
        lib.hdfs3x_stream_read_ex(ctx.ctx, dp[i % nb], bb, args.read_grid, sink.data_ptr(), int(overlap and i > 0))

    def settle():
        done = torch.cuda.Event()
        done.record(stream)
        while not done.query():
            pass
        torch.cuda.synchronize()

    def region(fn, pre, k):
        """pre(): whatever precedes the region; returns (us per launch, per-launch stamps)"""
        lib.hdfs3x_clock_stamps(None, 0)
        pre()
        torch.cuda.synchronize()
        stamps.zero_()
        lib.hdfs3x_clock_stamps(stamps.data_ptr(), cap)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for i in range(k):
            fn(i, True)
        b.record(stream)
        torch.cuda.synchronize()
        n = lib.hdfs3x_clock_stamps(None, 0)
        st = stamps[:4 * min(n, cap)].view(-1, 4).cpu().numpy().astype(np.float64)
        st = st[np.argsort(st[:, 1])]
        mhz = 100.0 * (st[:, 2] - st[:, 0]) / np.maximum(st[:, 3] - st[:, 1], 1)
        r0 = st[0, 1] if len(st) else 0
        starts = (st[:, 1] - r0) / 100.0  # us
        return a.elapsed_time(b) * 1e3 / k, mhz, starts

    out = []
    K, W = args.k, args.w
    for rep in range(args.reps):
        kinds = {"crc": crc_launch, "compute": compute_launch, "read": read_launch}
        for kind in args.kinds.split(","):
            fn = kinds[kind]
            lib.hdfs3x_set_variant(0 if kind == "read" else 125)

            def pre_bench():
                for i in range(2000):
                    fn(i, False)
                for i in range(W):
                    fn(i, True)
                settle()

            def pre_steady():
                for i in range(50):
                    fn(i, True)
                settle()

            def pre_busy():
                for i in range(W):
                    fn(i, True)
                torch.cuda._sleep(int(args.spin_us * cycles_per_us))

            def pre_queued():
                for i in range(500):
                    fn(i, True)

            for phase, pre, k in (("bench", pre_bench, K), ("steady", pre_steady, max(K, 200)),
                                  ("busy", pre_busy, K), ("queued", pre_queued, K)):
                if phase not in args.phases.split(","):
                    continue
                if phase in ("busy", "queued"):
                    # no host sync between pre() and the region: region() syncs after pre(), so inline
                    lib.hdfs3x_clock_stamps(None, 0)
                    torch.cuda.synchronize()
                    for i in range(300):  # sustained load first, as in the bench's pre-passes
                        fn(i, True)
                    stamps.zero_()
                    lib.hdfs3x_clock_stamps(stamps.data_ptr(), cap)
                    pre()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(stream)
                    for i in range(k):
                        fn(i, True)
                    b.record(stream)
                    torch.cuda.synchronize()
                    n = lib.hdfs3x_clock_stamps(None, 0)
                    st = stamps[:4 * min(n, cap)].view(-1, 4).cpu().numpy().astype(np.float64)
                    st = st[np.argsort(st[:, 1])][-k:]  # the region's own launches
                    mhz = 100.0 * (st[:, 2] - st[:, 0]) / np.maximum(st[:, 3] - st[:, 1], 1)
                    starts = (st[:, 1] - st[0, 1]) / 100.0
                    us = a.elapsed_time(b) * 1e3 / k
                else:
                    us, mhz, starts = region(fn, pre, k)
                s2s = np.diff(starts)
                out.append({"rep": rep, "kind": kind, "phase": phase, "k": k, "us_per_launch": round(us, 2),
                            "mhz_first10": [int(x) for x in mhz[:10]], "mhz_median": int(np.median(mhz)) if len(mhz) else 0,
                            "mhz_last5": [int(x) for x in mhz[-5:]],
                            "s2s_first10": [round(float(x), 2) for x in s2s[:10]],
                            "s2s_median": round(float(np.median(s2s)), 2) if len(s2s) else 0,
                            "stamps": int(len(mhz))})
                print(json.dumps(out[-1]), flush=True)
    lib.hdfs3x_set_variant(0)
    lib.hdfs3x_clock_stamps(None, 0)
    assert not bool((res != 0).any().item()), "clean blocks reported bad"


if __name__ == "__main__":
    main()
