#!/usr/bin/env python3
"""A/B of the segmented kernel's non-uniform segment lookup on 1 GiB of blocks:
  v0   binary-search loop (production before this A/B)
  v51  fixed-depth unrolled search (no loop in the hot loop's CFG)
Cases: 8 ragged blocks (chunk-aligned cuts that are not whole rounds, so the host finds
no uniform size) and, as the reference point, 8 equal 128 MiB blocks (UNI view), each in
verify and compute mode at bpc 512. Parity first: compute words equal the contiguous
kernel's, a clean verify reports nothing, and a flipped bit is found at its (block,
chunk). HIP-event timed, interleaved rounds, median us per launch. One JSON line."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    var = int(sys.argv[1]) if len(sys.argv) > 1 else 51
    lib = _native.lab()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx = CrcContext(0, lib=_native.lab())
    ctx.set_stream(st.cuda_stream)
    nb, bb, bpc = 8, 128 << 20, 512
    total = nb * bb
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    ref = torch.empty(4 * (total // bpc), dtype=torch.uint8, device=dev)
    ctx.compute_dev(data.data_ptr(), total, bpc, ref.data_ptr())
    out = torch.zeros_like(ref)
    res = torch.zeros(1024, dtype=torch.int64, device=dev)
    base = data.data_ptr()

    def mk(crc_base, layout):
        if layout == "ragged":    # unequal sizes, starts 512 B past a 4 KiB boundary
            cuts = [0] + [b * bb + (b * 37 % 7 + 1) * bpc for b in range(1, nb)] + [total]
        elif layout == "ragged4k":  # unequal sizes, every start 4 KiB aligned
            cuts = [0] + [b * bb + (b * 37 % 7 + 1) * 4096 for b in range(1, nb)] + [total]
        elif layout == "shifted":   # equal sizes (uniform view), every start 512 B past 4 KiB
            cuts = [0] + [b * bb + bpc for b in range(1, nb)] + [total]
        else:
            cuts = [b * bb for b in range(nb)] + [total]
        return [(base + cuts[i], crc_base + 4 * (cuts[i] // bpc), cuts[i + 1] - cuts[i]) for i in range(nb)], cuts

    layouts = {k: k for k in (["ragged", "ragged4k", "shifted", "equal"] if var == 0 else ["ragged", "equal"])}
    parity = {}
    for v in sorted({0, var}):
        lib.hdfs3x_set_variant(v)
        for name, rg in layouts.items():
            blocks_out, _ = mk(out.data_ptr(), rg)
            out.zero_()
            ctx.compute_blocks_dev(blocks_out, bpc)
            torch.cuda.synchronize()
            parity[f"compute_{name}_v{v}"] = bool(torch.equal(out, ref))
            blocks_ref, cuts = mk(ref.data_ptr(), rg)
            clean = ctx.verify_blocks_dev(blocks_ref, bpc) == (-1, -1)
            pos = cuts[5] + 3 * 4096 * 1000 + 777  # inside block 5
            data[pos] ^= 1
            got = ctx.verify_blocks_dev(blocks_ref, bpc)
            data[pos] ^= 1
            parity[f"verify_{name}_v{v}"] = clean and got == (5, (pos - cuts[5]) // bpc)
        lib.hdfs3x_set_variant(0)
    if not all(parity.values()):
        print(json.dumps({"bench": "seg_search_ab", "parity": parity}))
        raise SystemExit("PARITY FAILURE")

    cases = {}
    for v in sorted({0, var}):
        for name, rg in layouts.items():
            bv, _ = mk(ref.data_ptr(), rg)
            bc, _ = mk(out.data_ptr(), rg)

            def fv(i, v=v, bv=bv):
                lib.hdfs3x_set_variant(v)
                ctx.verify_blocks_dev_async(bv, bpc, res.data_ptr() + 8 * (i % 1024))
                lib.hdfs3x_set_variant(0)

            def fc(i, v=v, bc=bc):
                lib.hdfs3x_set_variant(v)
                ctx.compute_blocks_dev(bc, bpc)
                lib.hdfs3x_set_variant(0)

            cases[f"verify_{name}_v{v}"] = fv
            cases[f"compute_{name}_v{v}"] = fc
    for f in cases.values():  # ramp
        for i in range(20):
            f(i)
    torch.cuda.synchronize()
    samples = {k: [] for k in cases}
    for _ in range(7):
        for name, f in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(5):
                f(i)
            e1.record(st)
            torch.cuda.synchronize()
            samples[name].append(e0.elapsed_time(e1) * 200)  # us per launch
    assert int(res.abs().sum()) == 0
    alg = (total // bpc) * (bpc + 4)
    print(json.dumps({"bench": "seg_search_ab", "variant": var, "parity": parity,
                      **{k: {"us_med": round(statistics.median(v), 2),
                             "TBps": round(alg / statistics.median(v) / 1e6, 3)} for k, v in samples.items()}}))


if __name__ == "__main__":
    main()
