#!/usr/bin/env python3
"""Probe (round 5): the bpc-65536 chain failure isolated. Arena 3 of tools/pieces_race_probe.py (96 packets
of 64 KiB, the last 65,236 B, words 4 B so the data sits at offset 36: not 16-B aligned, so the stream
API falls back to descriptors and the chunk-per-lane packet kernel) verified alone, repeatedly, through
the stream API and the synchronous descriptor API, barriered; then after one launch over a full-last-packet
arena. One JSON line per case: the keys reported."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]


def main():
    import numpy as np
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext, DeviceBuffer
    from test_gpu_packet_stream import build_arena

    ctx = CrcContext(0)
    bpc, n, plen = 65536, 96, 65536
    h3, pitch, crc_off, data_off, datas = build_arena(n, plen, plen - 300, bpc, 7000 + 131 * 3 + bpc % 1013)
    h0, _, _, _, _ = build_arena(n, plen, plen, bpc, 7000 + bpc % 1013)
    d3, d0 = ctx.upload(h3), ctx.upload(h0)
    s3 = CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, plen - 300)
    s0 = CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, plen)
    res = DeviceBuffer(8 * 64)
    print(json.dumps({"data_off": data_off, "pitch": pitch, "aligned16": (d3.ptr + data_off) % 16 == 0}), flush=True)

    def keys(nl):
        w = ctx.download(res, 8 * nl).view(np.uint64).tolist()
        return [None if x == 0 else [ctx.decode_result(int(x)) >> 32, ctx.decode_result(int(x)) & 0xFFFFFFFF] for x in w]

    for name, seq in [("arena3_alone", [3] * 12), ("alt_0_3", [0, 3] * 6), ("after_0", [0, 3, 3, 3, 3, 3])]:
        ctx.memset(res, 0, 8 * 64)
        for i, a in enumerate(seq):
            d, s, h = (d3, s3, h3) if a == 3 else (d0, s0, h0)
            ctx.verify_packet_stream_async(d.ptr, h.nbytes, s, bpc, res.ptr + 8 * i)
            ctx.synchronize()  # one launch at a time
        print(json.dumps({"case": name, "seq": seq, "keys": keys(len(seq))}), flush=True)
    pk = [(i * pitch + data_off, i * pitch + crc_off, plen if i + 1 < n else plen - 300) for i in range(n)]
    print(json.dumps({"case": "sync_descriptors_arena3",
                      "keys": [ctx.verify_packets_dev(d3.ptr, h3.nbytes, pk, bpc, False) for _ in range(6)]}), flush=True)


if __name__ == "__main__":
    main()
