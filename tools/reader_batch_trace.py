#!/usr/bin/env python3
"""The block reader's GPU batches against contiguous 4 MiB verifies, for a kernel trace (VERDICT r4
item 4: "a kernel trace of a 64-packet batch shows the block-walk kernel at the 4 MiB contiguous time").

  run        (under rocprofv3 --kernel-trace) phase 1: `--mib` of 64 KiB packets read through
             hdfs3_block_reader from the loopback datanode, `--reps` times, verify on, 64-packet batches
             (the reader's default; layout from --layout: dense = round 5's default, wire = the
             HDFS3_READER_LAYOUT=wire knob); one compute launch as a separator; phase 2: 200 barriered
             contiguous verifies of 4 MiB blocks resident in HBM, rotating over 16 (the same payload shape).
  summarize  <run_kernel_trace.csv>: the verify kernels of each phase (name, count, mean / median
             duration), split at the separator; one JSON line.

    rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/reader_batch_trace.py run --layout dense
    python3 tools/reader_batch_trace.py summarize out/.../run_kernel_trace.csv
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]


def run(args):
    os.environ["HDFS3_READER_LAYOUT"] = args.layout  # read once by the library, at its first reader
    import numpy as np
    import torch
    from libhdfs3_amd.engine import BlockReader, CrcContext
    from loopback import LoopbackDatanode

    dev = torch.device("cuda", 0)
    n = args.mib << 20
    host = np.random.default_rng(5).integers(0, 256, n, dtype=np.uint8)
    ctx = CrcContext(0)
    crc = ctx.compute(host, 512)
    dn = LoopbackDatanode(packet_bytes=65536)
    try:
        dn.add_block(1, host, crc, 512)
        out = np.empty(n, np.uint8)
        for _ in range(args.reps):
            with BlockReader("127.0.0.1", dn.port, 1, 0, n, batch_packets=64) as r:
                pos = 0
                while pos < n:
                    got = r.read_into(out, pos, min(4 << 20, n - pos))
                    assert got > 0
                    pos += got
            assert np.array_equal(out, host)
    finally:
        dn.stop()
    # separator: one compute launch (a kernel name no verify has)
    blocks = torch.randint(0, 256, (16, 4 << 20), dtype=torch.uint8, device=dev)
    words = torch.empty((16, (4 << 20) // 512 * 4), dtype=torch.uint8, device=dev)
    for b in range(16):
        ctx.compute_dev(blocks[b].data_ptr(), 4 << 20, 512, words[b].data_ptr())
    ctx.synchronize()
    res = torch.zeros(256, dtype=torch.int64, device=dev)
    for i in range(200):
        ctx.verify_dev_async(blocks[i % 16].data_ptr(), 4 << 20, 512, words[i % 16].data_ptr(),
                             res.data_ptr() + 8 * (i % 256))
    ctx.synchronize()
    assert not bool((res != 0).any().item())
    print(json.dumps({"layout": args.layout, "read_mib": args.mib, "reps": args.reps, "ok": True}), flush=True)


def summarize(args):
    path = args.csv
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur, seen_sep = [[], []], 0, False
    for r in rows:
        name = r["Kernel_Name"]
        if "crc32c_" not in name:
            continue
        m = re.search(r"(crc32c_\w+)<([^>]*)>", name)
        short = f"{m.group(1)}<{m.group(2)}>" if m else name[:80]
        verify = bool(re.search(r"<\s*\d+,\s*true", short))
        if not verify:  # compute launches: the .meta words before phase 1, the separator before phase 2
            if phases[0]:
                seen_sep = True
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        phases[1 if seen_sep else 0].append((short, d))
    out = {"trace": path}
    for label, ph in zip(("reader_batches", "contiguous_4mib"), phases):
        by = {}
        for k, d in ph:
            by.setdefault(k, []).append(d)
        out[label] = {k: {"n": len(v), "mean_us": round(statistics.mean(v), 2),
                          "median_us": round(statistics.median(v), 2)} for k, v in by.items()}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--layout", choices=["dense", "wire"], default="dense")
    r.add_argument("--mib", type=int, default=256)
    r.add_argument("--reps", type=int, default=3)
    s = sub.add_parser("summarize")
    s.add_argument("csv")
    args = ap.parse_args()
    run(args) if args.cmd == "run" else summarize(args)


if __name__ == "__main__":
    main()
