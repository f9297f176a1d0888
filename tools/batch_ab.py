#!/usr/bin/env python3
"""Multi-block batch API A/B (docs/DESIGN_HISTORY.md §4.2): 8 x 128 MiB device-resident blocks per call
through hdfs3_crc32c_verify_blocks_dev_async, with the wave kernel's pitch mode for blocks at constant strides (variant 0)
and with the segmented kernel forced (variant 54), against one contiguous 1 GiB verify of the
same bytes. HIP events on one stream, rounds interleaved; medians per case."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    extra = [int(v) for v in sys.argv[sys.argv.index("--variants") + 1].split(",")] if "--variants" in sys.argv else []
    lib = _native.lab()
    ctx = CrcContext(0, lib=lib)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    bpc, nb, bs = 512, 8, 128 << 20
    big = torch.randint(0, 256, (nb * bs,), dtype=torch.uint8, device="cuda")
    words = torch.zeros(nb * bs // bpc * 4, dtype=torch.uint8, device="cuda")
    sep = [torch.randint(0, 256, (bs,), dtype=torch.uint8, device="cuda") for _ in range(nb)]
    sepw = [torch.zeros(bs // bpc * 4, dtype=torch.uint8, device="cuda") for _ in range(nb)]
    ctx.compute_dev(big.data_ptr(), big.numel(), bpc, words.data_ptr())
    for d, w in zip(sep, sepw):
        ctx.compute_dev(d.data_ptr(), bs, bpc, w.data_ptr())
    res = torch.zeros(1, dtype=torch.int64, device="cuda")
    sliced = [(big.data_ptr() + i * bs, words.data_ptr() + i * (bs // bpc * 4), bs) for i in range(nb)]
    separate = [(d.data_ptr(), w.data_ptr(), bs) for d, w in zip(sep, sepw)]
    torch.cuda.synchronize()

    def timed(fn, reps=20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    cases = {
        "contiguous_1GiB": lambda: ctx.verify_dev_async(big.data_ptr(), big.numel(), bpc, words.data_ptr(),
                                                        res.data_ptr()),
        "blocks_sliced_v0": lambda: ctx.verify_blocks_dev_async(sliced, bpc, res.data_ptr()),
        "blocks_separate_v0": lambda: ctx.verify_blocks_dev_async(separate, bpc, res.data_ptr()),
    }
    for _ in range(200):
        cases["contiguous_1GiB"]()
    torch.cuda.synchronize()
    samples = {k: [] for k in list(cases) + ["blocks_sliced_v54", "blocks_separate_v54"]}
    for _ in range(7):
        for name, fn in cases.items():
            samples[name].append(timed(fn))
        lib.hdfs3x_set_variant(54)
        samples["blocks_sliced_v54"].append(timed(cases["blocks_sliced_v0"]))
        samples["blocks_separate_v54"].append(timed(cases["blocks_separate_v0"]))
        for v in extra:  # other lab variants over every case (pitch walk, segments, contiguous)
            lib.hdfs3x_set_variant(v)
            for name, fn in cases.items():
                samples.setdefault(name.replace("_v0", "") + f"_v{v}", []).append(timed(fn))
        lib.hdfs3x_set_variant(0)
    assert int(res.item()) == 0, "clean blocks reported a bad chunk"
    for name, v in samples.items():
        v.sort()
        print(json.dumps({"bench": "batch_ab", "case": name, "us_med": round(v[len(v) // 2], 2),
                          "us_min": round(v[0], 2), "GiBps_med": round(nb * bs / 2**30 / (v[len(v) // 2] * 1e-6), 1)}),
              flush=True)


if __name__ == "__main__":
    main()
