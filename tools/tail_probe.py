#!/usr/bin/env python3
"""Cost of a ragged end on the contiguous API (wave kernel): verify and compute of 1 GiB
at bpc 512 against the same plus 7 whole chunks and a 300-byte short tail (the wave
kernel's slow region: one lane per leftover chunk). HIP-event timed, median us per launch
of 5 interleaved rounds x 5 launches. One JSON line."""
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
    bpc, base_len = 512, 1 << 30
    lens = {"whole": base_len, "ragged": base_len + 7 * bpc + 300}
    buf = torch.randint(0, 256, (lens["ragged"],), dtype=torch.uint8, device=dev)
    crc = torch.empty(4 * ((lens["ragged"] + bpc - 1) // bpc), dtype=torch.uint8, device=dev)
    out = torch.empty_like(crc)
    ctx.compute_dev(buf.data_ptr(), lens["ragged"], bpc, crc.data_ptr())
    res = torch.zeros(1024, dtype=torch.int64, device=dev)
    cases = {}
    for name, n in lens.items():
        assert ctx.verify_dev(buf.data_ptr(), n, bpc, crc.data_ptr(), True) == -1
        cases[f"verify_{name}"] = (lambda i, n=n: ctx.verify_dev_async(buf.data_ptr(), n, bpc, crc.data_ptr(),
                                                                      res.data_ptr() + 8 * (i % 1024)))
        cases[f"compute_{name}"] = (lambda i, n=n: ctx.compute_dev(buf.data_ptr(), n, bpc, out.data_ptr()))
    for f in cases.values():
        for i in range(20):
            f(i)
    torch.cuda.synchronize()
    assert torch.equal(out, crc)
    samples = {k: [] for k in cases}
    for _ in range(5):
        for name, f in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(5):
                f(i)
            e1.record(st)
            torch.cuda.synchronize()
            samples[name].append(e0.elapsed_time(e1) * 200)
    assert int(res.abs().sum()) == 0
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    print(json.dumps({"bench": "tail_probe", "build": tag, **{k: round(statistics.median(v), 2)
                                                              for k, v in samples.items()}}))


if __name__ == "__main__":
    main()
