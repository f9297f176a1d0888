#!/usr/bin/env python3
"""A/B of held CRC-word stores in the segmented kernel's compute mode (bpc 512): A/B
variant 50 (per-round stores, the kernel before held stores) against production (held
stores since this A/B; before it, the roles were reversed), on the same 1 GiB:
  blocks8      hdfs3_crc32c_compute_blocks_dev over 8 x 128 MiB blocks (UNI view)
  ragged       the same bytes as 8 blocks of unequal, non-round sizes (binary-search view)
  packets      1 GiB as 64 KiB packets in wire layout (hdfs3_crc32c_compute_packets_dev)
Parity first: every case's CRC words from both variants must be identical (and equal the
contiguous wave kernel's words for the same bytes). Then HIP-event timed, interleaved
rounds, median us per launch. One JSON line."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    var = int(sys.argv[1]) if len(sys.argv) > 1 else 50
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
    base, obase = data.data_ptr(), out.data_ptr()
    blocks8 = [(base + b * bb, obase + 4 * (b * bb // bpc), bb) for b in range(nb)]
    # ragged: cut points at chunk multiples but not round (4 KiB) multiples
    cuts = [0] + [b * bb + (b * 37 % 7 + 1) * bpc for b in range(1, nb)] + [total]
    ragged = [(base + cuts[i], obase + 4 * (cuts[i] // bpc), cuts[i + 1] - cuts[i]) for i in range(nb)]

    # packets: [crc region][data] per 64 KiB packet in one arena (wire layout of the reader)
    pdata = 64 << 10
    npk = total // pdata
    crc_per = 4 * (pdata // bpc)
    arena = torch.empty(npk * (crc_per + pdata), dtype=torch.uint8, device=dev)
    av = arena.view(npk, crc_per + pdata)
    av[:, crc_per:] = data.view(npk, pdata)
    pk = [(i * (crc_per + pdata) + crc_per, i * (crc_per + pdata), pdata) for i in range(npk)]

    def run_blocks(blocks, v):
        lib.hdfs3x_set_variant(v)
        ctx.compute_blocks_dev(blocks, bpc)
        lib.hdfs3x_set_variant(0)

    descs = ctx._descs(pk)  # built once: the timed calls measure the API, not Python

    def run_packets(v):
        lib.hdfs3x_set_variant(v)
        _native.check("hdfs3_crc32c_compute_packets_dev",
                      lib.hdfs3_crc32c_compute_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), descs,
                                                           len(pk), bpc))
        lib.hdfs3x_set_variant(0)

    parity = {}
    for v in (0, var):
        for name, blocks in (("blocks8", blocks8), ("ragged", ragged)):
            out.zero_()
            run_blocks(blocks, v)
            torch.cuda.synchronize()
            parity[f"{name}_v{v}"] = bool(torch.equal(out, ref))
        av[:, :crc_per] = 0
        run_packets(v)
        torch.cuda.synchronize()
        parity[f"packets_v{v}"] = bool(torch.equal(av[:, :crc_per].reshape(-1), ref))
    if not all(parity.values()):
        print(json.dumps({"bench": "seg_hold_ab", "parity": parity}))
        raise SystemExit("PARITY FAILURE")

    cases = {}
    for v in (0, var):
        cases[f"blocks8_v{v}"] = (lambda v=v: run_blocks(blocks8, v))
        cases[f"ragged_v{v}"] = (lambda v=v: run_blocks(ragged, v))
        cases[f"packets_v{v}"] = (lambda v=v: run_packets(v))
    for f in cases.values():  # ramp
        for _ in range(20):
            f()
    torch.cuda.synchronize()
    samples = {k: [] for k in cases}
    for _ in range(7):
        for name, f in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                f()
            e1.record(st)
            torch.cuda.synchronize()
            samples[name].append(e0.elapsed_time(e1) * 200)  # us per launch
    alg = (total // bpc) * (bpc + 4)
    print(json.dumps({"bench": "seg_hold_ab", "variant": var, "parity": parity,
                      **{k: {"us_med": round(statistics.median(v), 2),
                             "TBps": round(alg / statistics.median(v) / 1e6, 3)} for k, v in samples.items()}}))


if __name__ == "__main__":
    main()
