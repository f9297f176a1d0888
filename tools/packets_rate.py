#!/usr/bin/env python3
"""Device-resident packet-stream verify/compute rate (hdfs3_crc32c_{verify,compute}_packets_dev):
1 GiB arena of 64 KiB packets in the wire layout [CRCs][data] (data 16 B aligned), the
segmented wave kernel (variant 0: constant-pitch packets take the descriptor-free strided
launch; variant 52: the same kernel with a descriptor array) vs the chunk-per-lane packet
kernel (variant 17). Each call includes the host-side descriptor pass and a stream sync
(the API is synchronous)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    ctx = CrcContext(0, lib=_native.lab())
    bpc, pkt = 512, 65536
    n = (1 << 30) // pkt
    stride = 512 + pkt  # [128 CRC words][64 KiB data]: data stays 16 B aligned
    arena = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device="cuda")
    desc = (_native.PktDesc * n)()
    for i in range(n):
        desc[i].data_off, desc[i].crc_off, desc[i].data_len, desc[i].reserved = i * stride + 512, i * stride, pkt, 0
    bp, bc = ctypes.c_int64(), ctypes.c_int64()
    out = []
    for v in (0, 52, 17, 0, 52):
        lib.hdfs3x_set_variant(v)
        _native.check("compute", lib.hdfs3_crc32c_compute_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n, bpc))
        _native.check("verify", lib.hdfs3_crc32c_verify_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n,
                                                                    bpc, 0, ctypes.byref(bp), ctypes.byref(bc)))
        assert bp.value == -1
        ts = {}
        for mode in ("verify", "compute"):
            t0 = time.perf_counter()
            reps = 10
            for _ in range(reps):
                if mode == "verify":
                    lib.hdfs3_crc32c_verify_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n, bpc, 0,
                                                        ctypes.byref(bp), ctypes.byref(bc))
                else:
                    lib.hdfs3_crc32c_compute_packets_dev(ctx.ctx, arena.data_ptr(), arena.numel(), desc, n, bpc)
            torch.cuda.synchronize()
            ts[mode] = (time.perf_counter() - t0) / reps
        out.append({"bench": "packets_dev", "variant": v, "packets": n, "packet_bytes": pkt,
                    "verify_GiBps": round(n * pkt / ts["verify"] / 2**30, 1),
                    "compute_GiBps": round(n * pkt / ts["compute"] / 2**30, 1)})
    lib.hdfs3x_set_variant(0)
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
