#!/usr/bin/env python3
"""Clock / power during sustained loads: is the 128 MiB verify launch rate set by the GPU's
clocks under its power limit?

Launch-level kernel traces of the driver's bench command (K=20 after an idle gap) show
single 128 MiB verifies at 19.2-19.7 us, the same-shape plain-read rate, while the same
launches sustained over thousands of steps average ~21 us. This tool runs phases of
back-to-back overlapped launches (verify kernel variants of the lab library, the plain-read
kernel: the same arena and launch shape as bench.py's ceiling), each `--seconds` long with idle gaps
between, and records
  * the per-launch time of every batch of 100 launches (HIP events), against time;
  * `amd-smi metric` samples (clocks, power) from a sampler thread, raw JSON per sample.
One JSON line per batch and per sample on stdout.

    python tools/clock_probe.py --seconds 3
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def sampler(stop, t0, out, period):
    cmds = [["amd-smi", "metric", "-g", "0", "--json"], ["rocm-smi", "-d", "0", "--showclocks", "--showpower", "--json"]]
    cmd = None
    for c in cmds:
        try:
            r = subprocess.run(c, capture_output=True, text=True, timeout=10)
            if r.returncode == 0 and r.stdout.strip():
                cmd = c
                break
        except Exception:
            continue
    if cmd is None:
        out.append({"smi": "unavailable"})
        return
    while not stop.is_set():
        ts = time.perf_counter() - t0
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=10)
            raw = r.stdout
            try:
                val = json.loads(raw)
            except Exception:
                val = raw[-4000:]
            out.append({"t": round(ts, 3), "t_end": round(time.perf_counter() - t0, 3), "tool": cmd[0], "smi": val})
        except Exception as e:  # noqa: BLE001 - recorded
            out.append({"t": round(ts, 3), "error": str(e)})
        stop.wait(period)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--idle", type=float, default=1.0)
    ap.add_argument("--period", type=float, default=0.1)
    ap.add_argument("--burst", type=int, default=100,
                    help="launches per HIP-event batch; with --gap-ms > 0 the GPU idles between batches")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="idle time between batches (duty-cycled load: average power below the limit)")
    ap.add_argument("--barriered", action="store_true", help="every verify launch keeps the AQL barrier bit")
    ap.add_argument("--phases", default="v0,read,v0",
                    help="comma list: vN = verify through the lab library with kernel variant N "
                         "(0 = production; diagnostic variants give wrong results on purpose), "
                         "read / readnt = the plain-read kernel, default / non-temporal loads")
    args = ap.parse_args()

    import torch
    import bench
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    dev = torch.device("cuda", 0)
    ctx = CrcContext(0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    work = bench.Workload(torch, ctx, dev, 128 << 20, 8, 512, seed=1234)
    lab = bench.lab_context(work, stream)
    lib = _native.lab()
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    result = torch.zeros(max(100, args.burst), dtype=torch.int64, device=dev)

    def verify_batch(i0, n):
        for i in range(n):
            b = (i0 + i) % work.blocks
            lab.verify_dev_async(work.data_ptr(b), work.block_bytes, 512, work.crc_ptr(b),
                                 result.data_ptr() + 8 * (i % result.numel()), overlap_previous=i > 0 and not args.barriered)

    def read_batch(i0, n, grid=256):
        for i in range(n):
            b = (i0 + i) % work.blocks
            lib.hdfs3x_stream_read_ex(lab.ctx, work.data_ptr(b), work.block_bytes, grid, sink.data_ptr(),
                                      int(i > 0 and not args.barriered))

    lines, samples = [], []
    stop = threading.Event()
    t0 = time.perf_counter()
    th = threading.Thread(target=sampler, args=(stop, t0, samples, args.period), daemon=True)
    th.start()
    time.sleep(args.idle)
    for k, phase in enumerate(args.phases.split(",")):
        fn = (read_batch if phase == "read" else
              (lambda i0, n: read_batch(i0, n, -256)) if phase == "readnt" else verify_batch)
        if not phase.startswith("read"):
            lib.hdfs3x_set_variant(int(phase[1:]))
        result.zero_()
        end = time.perf_counter() + args.seconds
        i = 0
        while time.perf_counter() < end:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn(i, args.burst)
            e1.record(stream)
            e1.synchronize()
            lines.append({"phase": phase, "k": k, "t": round(time.perf_counter() - t0, 4), "batch": i // args.burst,
                          "us_per_launch": round(e0.elapsed_time(e1) * 1e3 / args.burst, 3)})
            i += args.burst
            if args.gap_ms > 0:
                time.sleep(args.gap_ms * 1e-3)
        if phase == "v0" and bool((result != 0).any().item()):
            raise SystemExit("clean blocks reported bad")
        lib.hdfs3x_set_variant(0)
        time.sleep(args.idle)
    stop.set()
    th.join(timeout=15)
    for ln in lines:
        print(json.dumps(ln))
    for s in samples:
        print(json.dumps({"sample": s}))


if __name__ == "__main__":
    main()
