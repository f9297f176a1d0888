#!/usr/bin/env python3
"""Probe (round 5): chained overlapped verifies of packet streams at bpc = R x 4096 (the pitch walk's
piece compute + the packet-mode combine + the short-tail kernel), many chains, counting result slots
that differ from the oracle's answer. It found the descriptor staging ring of the packets API being
rewritten under a queued copy (arena 3 here: data off 16-byte alignment, so its stream takes the
descriptor path; 120 of 900 slots wrong before the fix, 0 after, with and without the piece compute
behind the AQL barrier (lab variant 155, removed); profiles/r05/r5d_*, r5f_*).

    python tools/pieces_race_probe.py --bpc 65536 --chains 20
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bpc", type=int, default=65536)
    ap.add_argument("--chains", type=int, default=20)
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--barriered", action="store_true", help="no HDFS3_LAUNCH_OVERLAP_PREVIOUS at all")
    args = ap.parse_args()
    import numpy as np
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext, DeviceBuffer
    from test_gpu_packet_stream import build_arena, oracle_key

    lib = _native.lab()
    ctx = CrcContext(0, lib=lib)
    bpc, n, plen = args.bpc, 96, 65536
    arenas, streams, hosts, want = [], [], [], []
    for a in range(5):
        last = plen if a != 3 else (bpc * 2 + 300 if bpc * 2 + 300 < plen else plen - 300)
        host, pitch, crc_off, data_off, datas = build_arena(n, plen, last, bpc, 7000 + 131 * a + bpc % 1013)
        if a == 2:
            host[61 * pitch + data_off + 40000] ^= 0x20
        hosts.append(host)
        arenas.append(ctx.upload(host))
        streams.append(CrcContext.packet_stream(crc_off, data_off, pitch, n, plen, last))
        k = oracle_key([np.frombuffer(host[i * pitch + data_off:i * pitch + data_off + datas[i].size], np.uint8)
                        for i in range(n)], host, pitch, crc_off, bpc, False)
        want.append(-1 if k == (-1, -1) else (k[0] << 32) | k[1])
    res = DeviceBuffer(args.launches * 8)
    for v in [int(x) for x in args.variants.split(",")]:
        lib.hdfs3x_set_variant(v)
        bad, examples = 0, []
        for c in range(args.chains):
            ctx.memset(res, 0, args.launches * 8)
            for i in range(args.launches):
                a = i % 5
                ctx.verify_packet_stream_async(arenas[a].ptr, hosts[a].nbytes, streams[a], bpc, res.ptr + 8 * i,
                                               overlap_previous=(i > 0 and not args.barriered))
            ctx.synchronize()
            words = ctx.download(res, args.launches * 8).view(np.uint64).tolist()
            for i, w in enumerate(words):
                got = ctx.decode_result(int(w)) if w else -1
                if got != want[i % 5]:
                    bad += 1
                    if len(examples) < 5:
                        examples.append({"chain": c, "launch": i, "arena": i % 5,
                                         "got": [got >> 32, got & 0xFFFFFFFF] if got >= 0 else -1})
        print(json.dumps({"variant": v, "bpc": bpc, "chains": args.chains, "launches": args.launches,
                          "barriered": args.barriered, "wrong_slots": bad, "examples": examples}), flush=True)
    lib.hdfs3x_set_variant(0)


if __name__ == "__main__":
    main()
