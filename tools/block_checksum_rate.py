"""Time the block checksum ("MD5 of CRC32", include/hdfs3_crc.h) on one 128 MiB block at
512 B chunks: hdfs3_block_checksum_dev (GPU CRC words + D2H + host MD5) against its host
MD5 alone (hdfs3_block_checksum_crcs over the same 1 MiB of words) and hashlib's MD5.
One JSON line per case; medians of `--reps` calls after 3 warm-ups."""
import argparse
import hashlib
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from libhdfs3_amd.engine import CrcContext, block_checksum_crcs  # noqa: E402


def med(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=128 << 20)
    ap.add_argument("--bpc", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, a.bytes, dtype=np.uint8)
    with CrcContext(0) as ctx:
        d = ctx.upload(data)
        crc = ctx.compute(data, a.bpc)
        md5, n = ctx.block_checksum_dev(d.ptr, a.bytes, a.bpc)
        assert md5 == hashlib.md5(crc.tobytes()).digest() == block_checksum_crcs(crc)
        t_dev = med(lambda: ctx.block_checksum_dev(d.ptr, a.bytes, a.bpc), a.reps)
    t_md5 = med(lambda: block_checksum_crcs(crc), a.reps)
    t_hashlib = med(lambda: hashlib.md5(crc.tobytes()).digest(), a.reps)
    base = {"block_bytes": a.bytes, "bpc": a.bpc, "crc_words": n}
    for case, t in (("hdfs3_block_checksum_dev", t_dev), ("hdfs3_block_checksum_crcs (host MD5 only)", t_md5),
                    ("hashlib.md5 of the words", t_hashlib)):
        print(json.dumps({**base, "case": case, "ms": round(t * 1e3, 3),
                          "block_GiBps": round(a.bytes / t / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
