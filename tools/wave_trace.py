#!/usr/bin/env python3
"""Per-wave timeline of the production verify kernel on a 128 MiB block (diagnostic
variant 13: the same kernel with s_memrealtime stamps, 100 MHz device-wide clock):
  t0 wave entry, t1 after the LDS table fill + barrier, t2 after the first step
  (first 2 rounds' data arrived and consumed), t3 end of the main loop.
Reports, per launch and as medians over launches: dispatch spread (t0 - min t0), fill
time, time to first step, and the distribution of wave end times — i.e. how much of a
launch is head (dispatch + first data), steady state and tail (imbalance).
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def pct(a, q):
    return round(float(np.percentile(a, q)), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=16)
    ap.add_argument("--bpc", type=int, default=512)
    ap.add_argument("--block-mib", type=int, default=128)
    ap.add_argument("--variant", type=int, default=13, help="13 = production + stamps, 15 = + s_setprio")
    ap.add_argument("--dump", default="", help="save the per-wave relative stamps (npz) of the first launches here")
    args = ap.parse_args()

    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(st)
    ctx = CrcContext(0, lib=_native.lab())
    ctx.set_stream(st.cuda_stream)
    blocks, bb = 8, args.block_mib << 20
    data = torch.randint(0, 256, (blocks, bb), dtype=torch.uint8, device=dev)
    nch = bb // args.bpc
    crc = torch.empty((blocks, 4 * nch), dtype=torch.uint8, device=dev)
    for b in range(blocks):
        ctx.compute_dev(data[b].data_ptr(), bb, args.bpc, crc[b].data_ptr())
    res = torch.zeros(blocks, dtype=torch.int64, device=dev)
    trace = torch.zeros(4096 * 16 * 4, dtype=torch.int64, device=dev)
    lib.hdfs3x_set_trace(trace.data_ptr())

    def launch(v, b):
        lib.hdfs3x_set_variant(v)
        ctx.verify_dev_async(data[b].data_ptr(), bb, args.bpc, crc[b].data_ptr(), res[b].data_ptr())

    for i in range(16):
        launch(0, i % blocks)
    torch.cuda.synchronize()
    # event-timed reference: production vs traced kernel, back to back
    ev = {}
    for v in (0, 14, args.variant):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(64):
            launch(v, i % blocks)
        e1.record(st)
        torch.cuda.synchronize()
        ev[v] = e0.elapsed_time(e1) * 1000 / 64
    rows, groups, raw = [], [], []
    for i in range(args.launches):
        trace.zero_()
        launch(args.variant, i % blocks)
        torch.cuda.synchronize()
        t = trace.cpu().numpy().reshape(-1, 4)
        t = t[t[:, 0] != 0]
        rel = (t - t[:, 0].min()) * 0.01  # 100 MHz ticks -> us
        rows.append({
            "waves": int(len(t)),
            "span_us": round(float(rel[:, 3].max()), 3),
            "dispatch_p50": pct(rel[:, 0], 50), "dispatch_max": pct(rel[:, 0], 100),
            "fill_p50": pct(rel[:, 1] - rel[:, 0], 50),
            "first_step_p50": pct(rel[:, 2], 50), "first_step_max": pct(rel[:, 2], 100),
            "end_p10": pct(rel[:, 3], 10), "end_p50": pct(rel[:, 3], 50), "end_p90": pct(rel[:, 3], 90),
            "end_max": pct(rel[:, 3], 100),
        })
        if len(t) == 4096:
            wid = np.arange(4096)
            blk = wid // 16
            if len(raw) < 4:
                raw.append(rel)
            wg_end = rel[:, 3].reshape(256, 16).max(axis=1)
            groups.append({
                # WGs go round-robin over the 8 XCDs: blockIdx % 8 (cdna_hip_programming.md)
                "end_by_xcd": [round(float(np.median(rel[blk % 8 == x, 3])), 2) for x in range(8)],
                "end_by_wave_in_wg": [round(float(np.median(rel[wid % 16 == w, 3])), 2) for w in range(16)],
                "end_by_blk_quartile": [round(float(np.median(rel[(blk // 64) == q, 3])), 2) for q in range(4)],
                "first_by_xcd": [round(float(np.median(rel[blk % 8 == x, 2])), 2) for x in range(8)],
                # per-CU (workgroup) completion: the last wave of each workgroup
                "cu_end_pcts": [pct(wg_end, q) for q in (0, 10, 50, 90, 100)],
                "cu_end_max_by_xcd": [round(float(wg_end[np.arange(256) % 8 == x].max()), 2) for x in range(8)],
            })
    lib.hdfs3x_set_variant(0)
    if args.dump and raw:
        np.savez_compressed(args.dump, rel=np.stack(raw))
    assert int(res.sum()) == 0, "verify reported a mismatch"
    med = {k: round(float(np.median([r[k] for r in rows])), 3) for k in rows[0]}
    print(json.dumps({"bench": "wave_trace", "bpc": args.bpc, "block_mib": args.block_mib,
                      "variant": args.variant,
                      "event_us_per_launch": {f"v{k}": round(v, 2) for k, v in ev.items()},
                      "median": med, "launches": rows[:4], "groups": groups[:4]}))


if __name__ == "__main__":
    main()
