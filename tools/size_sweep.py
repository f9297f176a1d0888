#!/usr/bin/env python3
"""Kernel time vs bytes per launch (fixed per-launch cost vs steady-state rate):
verify (variants), coalesced-read probe and the stream-read ceiling, 16 MiB..1 GiB,
each launch on a distinct region of a 2 GiB arena (rotating, past the MALL)."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,2").split(",")]
    lib = _native.lab()
    dev = torch.device("cuda", 0)
    ctx = CrcContext(0, lib=_native.lab())
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx.set_stream(st.cuda_stream)
    arena = 2 << 30
    bpc = 512
    data = torch.randint(0, 256, (arena,), dtype=torch.uint8, device=dev)
    crc = torch.empty(4 * (arena // bpc), dtype=torch.uint8, device=dev)
    lib.hdfs3x_set_variant(0)
    ctx.compute_dev(data.data_ptr(), arena, bpc, crc.data_ptr())
    sink = torch.zeros(16, dtype=torch.int32, device=dev)
    res = torch.zeros(4096, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    for mib in [int(x) for x in os.environ.get("SIZES", "16,32,64,128,256,512,1024").split(",")]:
        n = mib << 20
        regions = arena // n

        def verify(v):
            def f(i):
                lib.hdfs3x_set_variant(v)
                off = (i % regions) * n
                ctx.verify_dev_async(data.data_ptr() + off, n, bpc, crc.data_ptr() + off // bpc * 4,
                                     res.data_ptr() + 8 * (i % 4096))
            return f

        cases = [(f"verify_v{v}", verify(v)) for v in variants]
        if mib in (16, 128):
            for v in (9, 10, 11, 12):
                cases.append((f"fixed_v{v}", verify(v)))
        cases.append(("read_G8", lambda i: lib.hdfs3x_lane_read(
            ctx.ctx, data.data_ptr() + (i % regions) * n, n, 512 | (2 << 16), sink.data_ptr())))
        cases.append(("stream", lambda i: lib.hdfs3x_stream_read(
            ctx.ctx, data.data_ptr() + (i % regions) * n, n, 512, sink.data_ptr())))
        reps = max(4, min(64, (2048 >> 0) // mib))
        samples = {c: [] for c, _ in cases}
        for _, f in cases:
            for i in range(3):
                f(i)
        for _ in range(5):
            for c, f in cases:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    f(i)
                e1.record()
                torch.cuda.synchronize()
                samples[c].append(e0.elapsed_time(e1) * 1e3 / reps)
        for c, xs in samples.items():
            med = statistics.median(xs)
            print(json.dumps({"MiB": mib, "case": c, "us": round(med, 2), "GBps": round(n / med / 1e3, 1)}), flush=True)
    assert not bool((res != 0).any().item()), "verify reported a bad chunk"
    lib.hdfs3x_set_variant(0)


if __name__ == "__main__":
    main()
