#!/usr/bin/env python3
"""CPU submission cost vs GPU time per single-block verify launch: is a Python-driven
loop of hdfs3_crc32c_verify_dev_async launches bound by the host? Times the issue loop
(perf_counter, before any synchronize) and the whole region (HIP events), after W warmup."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx = CrcContext(0, lib=_native.lab())
    ctx.set_stream(st.cuda_stream)
    blocks, bb, bpc = 8, 128 << 20, 512
    data = torch.randint(0, 256, (blocks, bb), dtype=torch.uint8, device=dev)
    crc = torch.empty((blocks, 4 * (bb // bpc)), dtype=torch.uint8, device=dev)
    for b in range(blocks):
        ctx.compute_dev(data[b].data_ptr(), bb, bpc, crc[b].data_ptr())
    res = torch.zeros(4096, dtype=torch.int64, device=dev)
    dp = [data[b].data_ptr() for b in range(blocks)]
    cp = [crc[b].data_ptr() for b in range(blocks)]
    rp = res.data_ptr()
    fn = lib.hdfs3_crc32c_verify_dev_async
    out = []
    for label, call in (("engine_wrapper", lambda i: ctx.verify_dev_async(dp[i % 8], bb, bpc, cp[i % 8], rp + 8 * (i % 4096))),
                        ("raw_ctypes", lambda i: fn(ctx.ctx, dp[i % 8], bb, bpc, cp[i % 8], 0, rp + 8 * (i % 4096)))):
        for W, K in ((10, 200), (1000, 2000)):
            for i in range(W):
                call(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            t0 = time.perf_counter()
            for i in range(K):
                call(i)
            t_issue = time.perf_counter() - t0
            e1.record(st)
            torch.cuda.synchronize()
            gpu = e0.elapsed_time(e1) * 1e3 / K
            out.append({"path": label, "warmup": W, "steps": K, "cpu_issue_us_per_launch": round(t_issue * 1e6 / K, 2),
                        "gpu_us_per_launch": round(gpu, 2)})
    assert int(res.abs().sum()) == 0
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
