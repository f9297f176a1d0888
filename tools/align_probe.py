#!/usr/bin/env python3
"""Rate of device-resident verify against the data pointer's offset from a 4 KiB
boundary: 1 GiB at bpc 512 through the contiguous API (wave kernel) and as 8 blocks
through the batch API (segmented kernel), for offsets 0, 16, 128, 256, 512, 1024, 2048
and 3072 B. HIP-event timed, interleaved rounds, median us per launch. One JSON line."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd.engine import CrcContext

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx = CrcContext(0)
    ctx.set_stream(st.cuda_stream)
    total, bpc, nb = 1 << 30, 512, 8
    buf = torch.randint(0, 256, (total + 8192,), dtype=torch.uint8, device=dev)
    crc = torch.empty(4 * (total // bpc), dtype=torch.uint8, device=dev)
    res = torch.zeros(1024, dtype=torch.int64, device=dev)
    base = buf.data_ptr()
    assert base % 4096 == 0
    offsets = [0, 16, 128, 256, 512, 1024, 2048, 3072]
    cases = {}
    for off in offsets:
        p = base + off
        ctx.compute_dev(p, total, bpc, crc.data_ptr())
        bb = total // nb
        blocks = [(p + b * bb, crc.data_ptr() + 4 * (b * bb // bpc), bb) for b in range(nb)]
        assert ctx.verify_dev(p, total, bpc, crc.data_ptr()) == -1
        assert ctx.verify_blocks_dev(blocks, bpc) == (-1, -1)
        # crc words are per offset: keep one copy per case
        c = crc.clone()
        blocks = [(p + b * bb, c.data_ptr() + 4 * (b * bb // bpc), bb) for b in range(nb)]
        cases[f"contig_{off}"] = (lambda i, p=p, c=c: ctx.verify_dev_async(p, total, bpc, c.data_ptr(),
                                                                          res.data_ptr() + 8 * (i % 1024)), c)
        cases[f"blocks_{off}"] = (lambda i, bl=blocks: ctx.verify_blocks_dev_async(bl, bpc,
                                                                                  res.data_ptr() + 8 * (i % 1024)), c)
    for f, _ in cases.values():
        for i in range(20):
            f(i)
    torch.cuda.synchronize()
    samples = {k: [] for k in cases}
    for _ in range(5):
        for name, (f, _) in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(5):
                f(i)
            e1.record(st)
            torch.cuda.synchronize()
            samples[name].append(e0.elapsed_time(e1) * 200)
    assert int(res.abs().sum()) == 0
    print(json.dumps({"bench": "align_probe", "bytes": total, "bpc": bpc,
                      **{k: round(statistics.median(v), 2) for k, v in samples.items()}}))


if __name__ == "__main__":
    main()
