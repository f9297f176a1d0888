#!/usr/bin/env python3
"""In-process paired A/B of a block-reader environment knob that the library reads at each open
(e.g. HDFS3_READER_LAUNCHER): the config-5 file (8 x 128 MiB blocks, 512 B chunks, 64 KiB packets
from the loopback datanode) read with the knob off and on, pass by pass, so that box drift falls on
both alike. Lines: single-stream hdfsRead (4 MiB reads) and 8 concurrent preads (one block each),
verify on; per line the medians and the median of the per-pair ratios (on / off).

    python tools/reader_ab.py --knob HDFS3_READER_LAUNCHER --reps 8
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tools")]
GIB = 2**30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", required=True)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--block-mib", type=int, default=128)
    ap.add_argument("--verify", type=int, default=1)
    ap.add_argument("--modes", default="hdfsRead,parallel_pread")
    args = ap.parse_args()

    from e2e_read import pread_block
    from libhdfs3_amd.engine import CrcContext, InputStream
    from loopback import LoopbackDatanode

    bsz = args.block_mib << 20
    total = args.blocks * bsz
    ctx = CrcContext(0)
    data = np.random.default_rng(0x5EED).integers(0, 256, size=total, dtype=np.uint8)
    crc = ctx.compute(data, 512)
    dn = LoopbackDatanode(packet_bytes=65536)
    blocks = []
    for i in range(args.blocks):
        dn.add_block(10 + i, data[i * bsz:(i + 1) * bsz], crc[4 * (i * bsz // 512):4 * ((i + 1) * bsz // 512)], 512)
        blocks.append((10 + i, bsz))
    located = [(b, n, [("127.0.0.1", dn.port)]) for b, n in blocks]
    out = np.empty(total, np.uint8)
    verify = bool(args.verify)

    def one_stream():
        with InputStream(located, verify=verify, batch_packets=64) as s:
            pos = 0
            while pos < total:
                got = s.read_into(out, pos, min(4 << 20, total - pos))
                assert got > 0
                pos += got

    def eight_streams():
        errors = []
        th = [threading.Thread(target=pread_block, args=(blocks, dn.port, i, bsz, out[i * bsz:(i + 1) * bsz],
                                                         verify, 64, errors)) for i in range(args.blocks)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors

    try:
        for name, fn in (("hdfsRead", one_stream), ("parallel_pread", eight_streams)):
            if name not in args.modes.split(","):
                continue
            rates = {"0": [], "1": []}
            for rep in range(1 + args.reps):
                for val in ("0", "1"):
                    os.environ[args.knob] = val
                    out[::4096] = ~data[::4096]
                    t0 = time.perf_counter()
                    fn()
                    dt = time.perf_counter() - t0
                    assert np.array_equal(out, data)
                    if rep:  # the first pair is untimed (rings, contexts)
                        rates[val].append(total / dt / GIB)
            ratios = [b / a for a, b in zip(rates["0"], rates["1"])]
            print(json.dumps({"knob": args.knob, "mode": name, "verify": verify,
                              "streams": 1 if name == "hdfsRead" else args.blocks,
                              "off_gib_s_med": round(statistics.median(rates["0"]), 2),
                              "on_gib_s_med": round(statistics.median(rates["1"]), 2),
                              "on_over_off_med": round(statistics.median(ratios), 4),
                              "on_over_off_all": [round(r, 3) for r in ratios]}), flush=True)
    finally:
        os.environ.pop(args.knob, None)
        dn.stop()
        ctx.close()


if __name__ == "__main__":
    main()
