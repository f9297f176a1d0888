#!/usr/bin/env python3
"""Does a HIP graph shrink the per-launch gap of single-block verifies? K launches of
verify_dev_async over 8 rotating 128 MiB blocks: eager back-to-back vs captured into a
graph (torch.cuda.graph on the ctx stream; our library shares torch's HIP runtime when
torch is imported first) and replayed. Every launch still verifies one whole block."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd.engine import CrcContext

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx = CrcContext(0)
    ctx.set_stream(st.cuda_stream)
    blocks, bb, bpc = 8, 128 << 20, 512
    data = torch.randint(0, 256, (blocks, bb), dtype=torch.uint8, device=dev)
    crc = torch.empty((blocks, 4 * (bb // bpc)), dtype=torch.uint8, device=dev)
    for b in range(blocks):
        ctx.compute_dev(data[b].data_ptr(), bb, bpc, crc[b].data_ptr())
    res = torch.zeros(4096, dtype=torch.int64, device=dev)

    def launches(n, base=0):
        for i in range(n):
            b = (base + i) % blocks
            ctx.verify_dev_async(data[b].data_ptr(), bb, bpc, crc[b].data_ptr(), res.data_ptr() + 8 * ((base + i) % 4096))

    out = {}
    launches(16)
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        launches(256)
        torch.cuda.synchronize()
        out.setdefault("eager_us", []).append((time.perf_counter() - t0) / 256 * 1e6)
    for per_graph in (8, 64):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            launches(per_graph)
        g.replay()
        torch.cuda.synchronize()
        for rep in range(3):
            t0 = time.perf_counter()
            for _ in range(256 // per_graph):
                g.replay()
            torch.cuda.synchronize()
            out.setdefault(f"graph{per_graph}_us", []).append((time.perf_counter() - t0) / 256 * 1e6)
    assert int(res.abs().sum()) == 0
    print(json.dumps({"bench": "graph_probe", **{k: [round(x, 2) for x in v] for k, v in out.items()}}))


if __name__ == "__main__":
    main()
