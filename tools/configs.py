#!/usr/bin/env python3
"""BASELINE.json configs the bench line does not cover, GPU side (docs/DESIGN_HISTORY.md §5):
  config 0  one 64 KiB HDFS packet (128 x 512 B chunks): latency of a single verify through
            the host-buffer API (H2D + kernel + result) and the packets API; the reference CPU
            timing of the same packet is bench.py's cpu_baseline.config0_packet_us
  config 2  1 GiB synthetic stream, compute (write) and verify (read) at bpc 512 / 2048 / 4096,
            after a 200-launch ramp, HIP events around batches of 5 back-to-back launches (median
            of 10), plus the compute -> verify round trip and a flip
Prints one JSON line per measurement."""
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from libhdfs3_amd.engine import CrcContext

    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx = CrcContext(0)
    ctx.set_stream(st.cuda_stream)

    # ---- config 2: 1 GiB stream, bpc sweep -------------------------------------------
    n = 1 << 30
    data = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
    res = torch.zeros(64, dtype=torch.int64, device=dev)
    for bpc in (512, 2048, 4096):
        nch = n // bpc
        crc = torch.empty(4 * nch, dtype=torch.uint8, device=dev)
        times = {"compute": [], "verify": []}

        def launch(mode, i):
            if mode == "compute":
                ctx.compute_dev(data.data_ptr(), n, bpc, crc.data_ptr())
            else:
                ctx.verify_dev_async(data.data_ptr(), n, bpc, crc.data_ptr(), res.data_ptr() + 8 * (i % 64))

        launch("compute", 0)
        # the GPU needs ~25 ms of sustained load to leave its idle power state (docs/DESIGN_HISTORY.md §5):
        # ramp with back-to-back launches, then time batches of BATCH back-to-back launches
        BATCH = 5
        for mode in ("compute", "verify"):
            for i in range(200):
                launch(mode, i)
            for rep in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for i in range(BATCH):
                    launch(mode, i)
                e1.record(st)
                e1.synchronize()
                times[mode].append(e0.elapsed_time(e1) * 1e-3 / BATCH)
        assert int(res.abs().sum()) == 0, "round trip: verify of freshly computed words failed"
        pos = n // 3 + 5
        orig = int(data[pos].item())
        data[pos] = orig ^ 0x40
        torch.cuda.synchronize()
        first = ctx.verify_dev(data.data_ptr(), n, bpc, crc.data_ptr())
        data[pos] = orig
        torch.cuda.synchronize()
        assert first == pos // bpc, (first, pos // bpc)
        for mode in ("compute", "verify"):
            t = statistics.median(times[mode])
            alg = nch * (bpc + 4)  # verify: data + words read; compute: data read + words written
            print(json.dumps({"bench": "config2_stream", "bpc": bpc, "mode": mode, "bytes": n,
                              "us": round(t * 1e6, 1), "GiBps_payload": round(n / t / 2**30, 1),
                              "alg_TBps": round(alg / t / 1e12, 3), "frac_of_8TBps": round(alg / t / 8e12, 4),
                              "round_trip_ok": True}), flush=True)
        del crc

    # ---- config 0: one 64 KiB packet, latency ----------------------------------------
    pkt = np.random.default_rng(3).integers(0, 256, size=65536, dtype=np.uint8)
    words = ctx.compute(pkt, 512)
    arena = np.concatenate([words, pkt])
    desc = [(words.nbytes, 0, pkt.nbytes)]
    lat = {"host_verify": [], "packets_verify": []}
    for i in range(2000):
        t0 = time.perf_counter()
        assert ctx.verify(pkt, 512, words) == -1
        t1 = time.perf_counter()
        assert ctx.verify_packets(arena, desc, 512) == (-1, -1)
        t2 = time.perf_counter()
        lat["host_verify"].append(t1 - t0)
        lat["packets_verify"].append(t2 - t1)
    for k, v in lat.items():
        print(json.dumps({"bench": "config0_packet", "api": k, "packet_bytes": 65536,
                          "us_median": round(statistics.median(v[100:]) * 1e6, 1),
                          "us_p99": round(float(np.percentile(v[100:], 99)) * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
