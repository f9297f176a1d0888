#!/usr/bin/env python3
"""Where the bench's single-region compute number (`compute.overlapped`, K = 20 timed launches) loses
against its paired regions: the same region form with the timed launches' destination arrays prepared
differently. Per repetition, in order (medians over --reps):

  verify     value's form: PRE_PASS barriered verifies, W warmup, settle, K timed (the reference line)
  cur        bench.py compute_block: poison `out`, PRE_PASS + W into scratch, settle, K timed into `out`
  prepass    PRE_PASS barriered computes into `out`, then poison it, W into scratch, settle, K into `out`
  warm       PRE_PASS + W into `out` (no poison after them), settle, K into `out`

    python tools/compute_region_probe.py --reps 5
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--w", type=int, default=5)
    ap.add_argument("--prepass", type=int, default=2000)
    args = ap.parse_args()
    import torch
    import bench
    from libhdfs3_amd.engine import CrcContext

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx = CrcContext(0)
    ctx.set_stream(stream.cuda_stream)
    work = bench.Workload(torch, ctx, dev, 128 << 20, 8, 512, 1234)
    out = torch.full_like(work.crc, 0xA5)
    scratch = torch.empty_like(work.crc)
    res = torch.zeros(256, dtype=torch.int64, device=dev)
    dp, nb, bb = work._dp, work.blocks, work.block_bytes
    op = [out[b].data_ptr() for b in range(nb)]
    sp = [scratch[b].data_ptr() for b in range(nb)]

    def compute(n, overlap, dst):
        for i in range(n):
            ctx.compute_dev(dp[i % nb], bb, 512, dst[i % nb], overlap_previous=overlap and i > 0)

    def verify(n, overlap):
        for i in range(n):
            ctx.verify_dev_async(dp[i % nb], bb, 512, work.crc_ptr(i % nb), res.data_ptr() + 8 * (i % 256),
                                 overlap_previous=overlap and i > 0)

    def timed(fn):
        bench.settle(torch, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.k

    K, W, P = args.k, args.w, args.prepass
    t = {"verify": [], "cur": [], "prepass": [], "warm": []}
    for _ in range(args.reps):
        verify(P, False)
        verify(W, True)
        t["verify"].append(timed(lambda: verify(K, True)))

        out.fill_(0xA5)
        compute(P, False, sp)
        compute(W, True, sp)
        t["cur"].append(timed(lambda: compute(K, True, op)))

        compute(P, False, op)
        out.fill_(0xA5)
        compute(W, True, sp)
        t["prepass"].append(timed(lambda: compute(K, True, op)))

        compute(P, False, op)
        compute(W, True, op)
        t["warm"].append(timed(lambda: compute(K, True, op)))
    assert not bool((res != 0).any().item())
    v = statistics.median(t["verify"])
    for k, xs in t.items():
        m = statistics.median(xs)
        print(json.dumps({"case": k, "us_med": round(m, 3), "us_all": [round(x, 2) for x in xs],
                          "verify_over_case": round(v / m, 4)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
