#!/usr/bin/env python3
"""A/B of the segmented kernel against the contiguous wave kernel on the same 1 GiB:
  contiguous   hdfs3_crc32c_verify_dev_async over the 8 contiguous 128 MiB blocks
  blocks       hdfs3_crc32c_verify_blocks_dev_async, the same bytes as 8 independent blocks
  one_segment  the same API with the whole 1 GiB as ONE block (segmented kernel, 1 segment)
  ragged       the same bytes as 8 blocks of unequal lengths (binary-search segment walk)
HIP-event timed, interleaved rounds, median us per launch."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


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
    nb, bb, bpc = 8, 128 << 20, 512
    data = torch.randint(0, 256, (nb, bb), dtype=torch.uint8, device=dev)
    crc = torch.empty((nb, 4 * (bb // bpc)), dtype=torch.uint8, device=dev)
    ctx.compute_dev(data.data_ptr(), nb * bb, bpc, crc.data_ptr())
    res = torch.zeros(1024, dtype=torch.int64, device=dev)
    blocks = [(data[b].data_ptr(), crc[b].data_ptr(), bb) for b in range(nb)]

    def contiguous(i):
        ctx.verify_dev_async(data.data_ptr(), nb * bb, bpc, crc.data_ptr(), res.data_ptr() + 8 * (i % 1024))

    def blk(v):
        def f(i):
            lib.hdfs3x_set_variant(v)
            ctx.verify_blocks_dev_async(blocks, bpc, res.data_ptr() + 8 * (i % 1024))
            lib.hdfs3x_set_variant(0)
        return f

    one = [(data.data_ptr(), crc.data_ptr(), nb * bb)]

    def one_segment(i):
        ctx.verify_blocks_dev_async(one, bpc, res.data_ptr() + 8 * (i % 1024))

    # ragged: the same bytes as 8 blocks of unequal whole-round lengths (binary-search segment walk)
    cut = [0] + [b * bb + (b * 37 % 11 - 5) * 4096 * 16 for b in range(1, nb)] + [nb * bb]
    ragged = [(data.data_ptr() + cut[b], crc.data_ptr() + 4 * (cut[b] // bpc), cut[b + 1] - cut[b]) for b in range(nb)]

    def ragged_v(v):
        def f(i):
            lib.hdfs3x_set_variant(v)
            ctx.verify_blocks_dev_async(ragged, bpc, res.data_ptr() + 8 * (i % 1024))
            lib.hdfs3x_set_variant(0)
        return f

    cases = {"contiguous": contiguous, "blocks": blk(0), "one_segment": one_segment, "ragged": ragged_v(0)}
    samples = {k: [] for k in cases}
    for f in cases.values():  # ramp the clocks (docs/DESIGN_HISTORY.md §5: ~25 ms of load)
        for i in range(100):
            f(i)
    torch.cuda.synchronize()
    for rnd in range(7):
        for name, f in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(10):
                f(i)
            e1.record(st)
            torch.cuda.synchronize()
            samples[name].append(e0.elapsed_time(e1) * 100)  # us per launch
    assert int(res.abs().sum()) == 0
    alg = nb * (bb // bpc) * (bpc + 4)
    print(json.dumps({"bench": "seg_ab", **{k: {"us_med": round(statistics.median(v), 2),
                                                "TBps": round(alg / statistics.median(v) / 1e6, 3)}
                                            for k, v in samples.items()}}))


if __name__ == "__main__":
    main()
