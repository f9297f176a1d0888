#!/usr/bin/env python3
"""Kernel diagnostics on one GPU (not the driver's bench): HBM read ceiling, the CRC
kernel's access pattern alone, and verify/compute rates per bytes-per-checksum.
Prints one JSON object per measurement. Rates are payload GB/s (1e9) from HIP events
on the launch stream; each launch covers one 128 MiB block, rotating over 8 blocks."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    dev = torch.device("cuda", 0)
    ctx = CrcContext(0, lib=_native.lab())
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)
    blocks, bb = 8, 128 << 20
    data = torch.randint(0, 256, (blocks, bb), dtype=torch.uint8, device=dev)
    sink = torch.zeros(16, dtype=torch.int32, device=dev)
    res = torch.zeros(1024, dtype=torch.int64, device=dev)
    reps = int(os.environ.get("SWEEP_REPS", "40"))

    def timed(fn, nbytes):
        for r in range(3):
            fn(r)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(reps):
            fn(r)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e-3 / reps
        return {"us": round(t * 1e6, 2), "GBps": round(nbytes / t / 1e9, 1)}

    out = []
    total = blocks * bb
    for grid in (0, 256, 512, 1024, 4096):
        r = timed(lambda i: lib.hdfs3x_stream_read(ctx.ctx, data.data_ptr(), total, grid, sink.data_ptr()), total)
        out.append({"kernel": "stream_read_1GiB", "grid": grid or "default", **r})
    for bpc in (512, 2048, 4096):
        nch = bb // bpc
        crc = torch.empty((blocks, 4 * nch), dtype=torch.uint8, device=dev)
        for v in range(5):
            r = timed(lambda i: lib.hdfs3x_lane_read(ctx.ctx, data[i % blocks].data_ptr(), bb, bpc | (v << 16),
                                                     sink.data_ptr()), bb)
            out.append({"kernel": "lane_read", "variant": v, "bpc": bpc, **r})
        r = timed(lambda i: ctx.compute_dev(data[i % blocks].data_ptr(), bb, bpc, crc[i % blocks].data_ptr()), bb)
        out.append({"kernel": "compute", "bpc": bpc, **r})
        res.zero_()
        r = timed(lambda i: ctx.verify_dev_async(data[i % blocks].data_ptr(), bb, bpc, crc[i % blocks].data_ptr(),
                                                 res.data_ptr() + 8 * (i % 1024)), bb)
        out.append({"kernel": "verify", "bpc": bpc, "clean": bool((res == 0).all().item()), **r})
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
