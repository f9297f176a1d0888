#!/usr/bin/env python3
"""Where a 128 MiB launch's time goes, wave by wave (barriered launches at 0.87 of
the read kernel's per-block rate). Lane 0 of every wave of the stamping kernels (lab variant 125 =
production verify + LabClock, and the plain stream read) records its realtime start/end (100 MHz),
its shader clocks and its XCC (LabClock wave buffer, crc32c_device.h). Every wave carries its launch's
number (a kernel argument: no atomics in the stamping path). Per launch:
  gap        previous launch's last wave end -> this launch's first wave start
  ramp       first -> last wave start (dispatch)
  body       last wave start -> first wave end
  tail       first wave end -> last wave end
  span       first start -> last end
  xcc_end    per XCC: median wave end - launch start (the XCDs' imbalance)
Medians over the K launches of a region, barriered and overlapped.

    python tools/wave_spread.py [--k 40] [--kinds crc,read]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=40)
    ap.add_argument("--kinds", default="crc,read")
    ap.add_argument("--read-grid", type=int, default=-512)
    ap.add_argument("--variant", type=int, default=125)
    ap.add_argument("--form", default="", choices=["", "bench"],
                    help="bench: the driver's region (2000 barriered, W overlapped, settle, K timed: the first "
                         "barriered, the rest overlapped) against K launches after 1000 overlapped ones; "
                         "per-launch rows instead of medians (with --mid: each launch's head)")
    ap.add_argument("--w", type=int, default=5)
    ap.add_argument("--mid", action="store_true", help="variant 146: word 2 holds the fill-done and first-data "
                    "times of the wave (kLabMid) instead of its shader clocks")
    args = ap.parse_args()

    import numpy as np
    import torch
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext

    lib = _native.lab()
    dev = torch.device("cuda", 0)
    ctx = CrcContext(0, lib=lib)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    nb, bb, bpc = 8, 128 << 20, 512
    data = torch.randint(0, 256, (nb, bb), dtype=torch.uint8, device=dev)
    crc = torch.empty((nb, 4 * (bb // bpc)), dtype=torch.uint8, device=dev)
    for b in range(nb):
        ctx.compute_dev(data[b].data_ptr(), bb, bpc, crc[b].data_ptr())
    res = torch.zeros(8192, dtype=torch.int64, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    cap = 1 << 20
    stamps = torch.zeros(cap * 4, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    dp = [data[b].data_ptr() for b in range(nb)]
    cp = [crc[b].data_ptr() for b in range(nb)]
    rp = res.data_ptr()

    def crc_launch(i, overlap):
        ctx.verify_dev_async(dp[i % nb], bb, bpc, cp[i % nb], rp + 8 * (i % 8192), overlap_previous=overlap and i > 0)

    def read_launch(i, overlap):
        lib.hdfs3x_stream_read_ex(ctx.ctx, dp[i % nb], bb, args.read_grid, sink.data_ptr(), int(overlap and i > 0))

    def settle():
        done = torch.cuda.Event()
        done.record(stream)
        while not done.query():
            pass
        torch.cuda.synchronize()

    def region(fn, overlap, k):
        for i in range(2000):
            fn(i, overlap)
        settle()
        stamps.zero_()
        lib.hdfs3x_wave_stamps(stamps.data_ptr(), cap)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for i in range(k):
            fn(i, overlap)
        b.record(stream)
        torch.cuda.synchronize()
        n = lib.hdfs3x_wave_stamps(None, 0)
        st = stamps.view(-1, 4).cpu().numpy()
        return a.elapsed_time(b) * 1e3 / k, n, st

    if args.form == "bench":
        lib.hdfs3x_set_variant(args.variant)
        m21 = np.uint64(0x1FFFFF)

        def launches(pre, stamped_pre):
            # stamped_pre: the buffer goes in before pre() (no sync between pre() and the region; the
            # ring keeps the last 256 launches, the region's are the last K)
            if stamped_pre:
                torch.cuda.synchronize()
                stamps.zero_()
                torch.cuda.synchronize()
                lib.hdfs3x_wave_stamps(stamps.data_ptr(), cap)
                pre()
            else:
                pre()
                stamps.zero_()
                torch.cuda.synchronize()
                lib.hdfs3x_wave_stamps(stamps.data_ptr(), cap)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for i in range(args.k):
                crc_launch(i, True)
            b.record(stream)
            torch.cuda.synchronize()
            n = lib.hdfs3x_wave_stamps(None, 0)
            st = stamps.view(-1, 4).cpu().numpy()
            st = st[st[:, 1] != 0]
            seq = (st[:, 3].astype(np.uint64) >> np.uint64(52)).astype(np.int64)
            region = [(n - args.k + li) & 0xFFF for li in range(args.k)]
            st = st[np.isin(seq, region)]
            seq = (st[:, 3].astype(np.uint64) >> np.uint64(52)).astype(np.int64)
            rows = []
            t_first = st[:, 0].min() / 100.0
            for li, sq in enumerate(region):
                x = st[seq == sq]
                r0, r1 = x[:, 0] / 100.0, x[:, 1] / 100.0
                row = {"launch": li + 1, "start_us": round(r0.min() - t_first, 2), "span_us": round(r1.max() - r0.min(), 2),
                       "wave_end_p10_p90_us": [round(float(np.percentile(r1 - r0.min(), q)), 2) for q in (10, 90)]}
                if args.mid:
                    w2 = x[:, 2].astype(np.uint64)
                    row["fill_done_p50_us"] = round(float(np.median((w2 & m21).astype(np.float64))) / 100.0, 2)
                    row["first_data_p50_us"] = round(float(np.median(((w2 >> np.uint64(21)) & m21).astype(np.float64))) / 100.0, 2)
                rows.append(row)
            return a.elapsed_time(b) * 1e3 / args.k, rows

        def pre_bench():
            for i in range(2000):
                crc_launch(i, False)
            for i in range(args.w):
                crc_launch(i, True)
            settle()

        def pre_steady():
            for i in range(1000):
                crc_launch(i, True)

        for name, pre, sp in (("bench", pre_bench, False), ("steady_after_1000", pre_steady, True)):
            us, rows = launches(pre, sp)
            print(json.dumps({"form": name, "k": args.k, "us_per_launch_events": round(us, 2), "launches": rows}),
                  flush=True)
        lib.hdfs3x_set_variant(0)
        lib.hdfs3x_wave_stamps(None, 0)
        assert not bool((res != 0).any().item()), "clean blocks reported bad"
        return

    out = []
    for kind in args.kinds.split(","):
        fn = crc_launch if kind == "crc" else read_launch
        lib.hdfs3x_set_variant(args.variant if kind == "crc" else 0)
        for overlap in (False, True):
            us, n, st = region(fn, overlap, args.k)
            st = st[st[:, 1] != 0]  # stamped slots
            per = len(st) // max(n, 1)
            if n != args.k or per * n != len(st) or len(st) >= cap:
                print(json.dumps({"kind": kind, "overlap": overlap, "error": f"{len(st)} stamps, {n} launches"}))
                continue
            seq = (st[:, 3].astype(np.uint64) >> np.uint64(52)).astype(np.int64)
            st = st[np.lexsort((st[:, 0], seq))]  # by launch, then start
            r0 = st[:, 0].astype(np.float64) / 100.0  # us
            r1 = st[:, 1].astype(np.float64) / 100.0
            clk = st[:, 2].astype(np.float64)
            xcc = (st[:, 3] >> 32) & 0xF
            # the CU each wave ran on: XCC and HW_ID's cu/sh/se fields (bits 8-15)
            cu = (((st[:, 3] >> 32) & 0xF) << 8) | ((st[:, 3] >> 8) & 0xFF)
            cu_ends = {}  # CU -> [its last wave end - launch start, per launch]
            rows = {"gap": [], "ramp": [], "body": [], "tail": [], "span": [], "mhz": []}
            xcc_end = {x: [] for x in range(8)}
            prev_end = None
            for li in range(args.k):
                s = slice(li * per, (li + 1) * per)
                a0, a1 = r0[s].min(), r0[s].max()
                e0, e1 = r1[s].min(), r1[s].max()
                if prev_end is not None:
                    rows["gap"].append(a0 - prev_end)
                prev_end = e1
                rows["ramp"].append(a1 - a0)
                rows["body"].append(e0 - a1)
                rows["tail"].append(e1 - e0)
                rows["span"].append(e1 - a0)
                rows["mhz"].append(float(np.median(clk[s] / np.maximum((r1[s] - r0[s]) * 100.0, 1) * 100.0)))
                cs, ends = cu[s], r1[s] - a0
                order = np.argsort(cs, kind="stable")
                ucs, first_idx = np.unique(cs[order], return_index=True)
                for c_id, e in zip(ucs, np.maximum.reduceat(ends[order], first_idx)):
                    cu_ends.setdefault(int(c_id), []).append(float(e))
                for x in range(8):
                    m = xcc[s] == x
                    if m.any():
                        xcc_end[x].append(float(np.median(r1[s][m])) - a0)
            rec = {"kind": kind, "overlap": overlap, "k": args.k, "waves_per_launch": per,
                   "us_per_launch_events": round(us, 2)}
            for key, xs in rows.items():
                rec[key + ("_med" if key == "mhz" else "_us_med")] = round(float(np.median(xs)), 2) if xs else None
            rec["xcc_end_us_med"] = {x: round(float(np.median(v)), 2) for x, v in xcc_end.items() if v}
            # is a slow CU slow in every launch? the spread of the CUs' mean end over the launches
            # against the spread inside one launch (equal: the same CUs are late every time)
            full = [v for v in cu_ends.values() if len(v) == args.k]
            if full:
                mat = np.array(full)  # CUs x launches
                rec["cus"] = len(full)
                rec["cu_end_within_launch_p10_p90_us"] = [round(float(np.median(np.percentile(mat, q, axis=0))), 2)
                                                          for q in (10, 90)]
                rec["cu_mean_end_p10_p90_us"] = [round(float(np.percentile(mat.mean(axis=1), q)), 2) for q in (10, 90)]
                rec["cu_rank_corr_consecutive"] = round(float(np.median(
                    [np.corrcoef(mat[:, i], mat[:, i + 1])[0, 1] for i in range(args.k - 1)])), 3)
            if args.mid and kind == "crc":
                w2 = st[:, 2].astype(np.uint64)
                m21 = np.uint64(0x1FFFFF)
                fill = (w2 & m21).astype(np.float64) / 100.0
                first = ((w2 >> np.uint64(21)) & m21).astype(np.float64) / 100.0
                karg = ((w2 >> np.uint64(42)) & m21).astype(np.float64) / 100.0
                rec["kernargs_us_p10_p50_p90"] = [round(float(np.percentile(karg, q)), 2) for q in (10, 50, 90)]
                rec["fill_done_us_p10_p50_p90"] = [round(float(np.percentile(fill, q)), 2) for q in (10, 50, 90)]
                rec["first_data_us_p10_p50_p90"] = [round(float(np.percentile(first, q)), 2) for q in (10, 50, 90)]
                # from the launch's first wave start to every wave's first data
                lf = []
                for li in range(args.k):
                    sl = slice(li * per, (li + 1) * per)
                    lf.append(np.percentile(r0[sl] + first[sl] - r0[sl].min(), 90))
                rec["launch_start_to_first_data_p90_us_med"] = round(float(np.median(lf)), 2)
                rec.pop("mhz_med", None)
            wave_life = r1 - r0
            rec["wave_life_us_p10_p50_p90"] = [round(float(np.percentile(wave_life, q)), 2) for q in (10, 50, 90)]
            out.append(rec)
            print(json.dumps(rec), flush=True)
    lib.hdfs3x_set_variant(0)
    lib.hdfs3x_wave_stamps(None, 0)
    assert not bool((res != 0).any().item()), "clean blocks reported bad"


if __name__ == "__main__":
    main()
