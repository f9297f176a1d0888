#!/usr/bin/env python3
"""Soak test of overlapped verify launches (HDFS3_LAUNCH_OVERLAP_PREVIOUS): for R rounds,
corrupt one random byte of one random block (8 x 128 MiB resident), verify a chain of
`--chain` overlapped single-block launches over all blocks, and check that every launch
reports exactly its block's first bad chunk (the corrupted one) or clean; then restore.
The expected answers come from the corruption position alone (the clean blocks' stored
CRCs were written by the GPU compute path and cross-checked against the oracle once)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--chain", type=int, default=64)
    ap.add_argument("--bpc", type=int, default=512)
    args = ap.parse_args()
    import torch
    from libhdfs3_amd.engine import CrcContext
    from util import oracle_compute  # checker only

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx = CrcContext(0)
    ctx.set_stream(st.cuda_stream)
    nblk, bb, bpc = 8, 128 << 20, args.bpc
    data = torch.randint(0, 256, (nblk, bb), dtype=torch.uint8, device=dev)
    crc = torch.empty((nblk, 4 * (bb // bpc)), dtype=torch.uint8, device=dev)
    for b in range(nblk):
        ctx.compute_dev(data[b].data_ptr(), bb, bpc, crc[b].data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(crc[0].cpu().numpy(), oracle_compute(data[0].cpu().numpy(), bpc))
    res = torch.zeros(args.chain, dtype=torch.int64, device=dev)
    rng = np.random.default_rng(0x50AC)
    t0, launches, failures = time.time(), 0, 0
    for r in range(args.rounds):
        blk = int(rng.integers(nblk))
        pos = int(rng.integers(bb))
        bit = 1 << int(rng.integers(8))
        data[blk, pos] ^= bit
        res.zero_()
        for i in range(args.chain):
            b = i % nblk
            ctx.verify_dev_async(data[b].data_ptr(), bb, bpc, crc[b].data_ptr(), res.data_ptr() + 8 * i,
                                 overlap_previous=i > 0)
        words = res.cpu().numpy().view(np.uint64)
        for i in range(args.chain):
            got = ctx.decode_result(int(words[i]))
            want = pos // bpc if i % nblk == blk else -1
            if got != want:
                failures += 1
                print(json.dumps({"round": r, "launch": i, "block": i % nblk, "got": got, "want": want}), flush=True)
        data[blk, pos] ^= bit
        launches += args.chain
    torch.cuda.synchronize()
    print(json.dumps({"soak": "overlapped_verify", "rounds": args.rounds, "launches": launches,
                      "failures": failures, "seconds": round(time.time() - t0, 1)}), flush=True)
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
