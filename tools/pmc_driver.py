#!/usr/bin/env python3
"""Small fixed workload for rocprofv3 PMC passes: `--launches` verify launches over
rotating 128 MiB blocks (8 blocks), kernel variant `--variant`."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bpc", type=int, default=512)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--launches", type=int, default=16)
    ap.add_argument("--mode", default="verify")
    ap.add_argument("--overlap", action="store_true",
                    help="launches after the first overlap their predecessor (the bench's timed mode)")
    args = ap.parse_args()
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    ctx = CrcContext(0, lib=_native.lab())
    dev = torch.device("cuda", 0)
    blocks, bb = 8, 128 << 20
    data = torch.randint(0, 256, (blocks, bb), dtype=torch.uint8, device=dev)
    crc = torch.empty((blocks, 4 * (bb // args.bpc)), dtype=torch.uint8, device=dev)
    res = torch.zeros(256, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    for b in range(blocks):
        ctx.compute_dev(data[b].data_ptr(), bb, args.bpc, crc[b].data_ptr())
    ctx.synchronize()
    lib.hdfs3x_set_variant(args.variant)
    for i in range(args.launches):
        if args.mode == "verify":
            ctx.verify_dev_async(data[i % blocks].data_ptr(), bb, args.bpc, crc[i % blocks].data_ptr(),
                                 res.data_ptr() + 8 * i, overlap_previous=args.overlap and i > 0)
        else:
            ctx.compute_dev(data[i % blocks].data_ptr(), bb, args.bpc, crc[i % blocks].data_ptr())
    ctx.synchronize()


if __name__ == "__main__":
    main()
