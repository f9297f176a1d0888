#!/usr/bin/env python3
"""From a rocprofv3 kernel-trace CSV: per-kernel average duration (start->end) and average
dispatch interval (start->start of consecutive dispatches of the same kernel) over its
longest back-to-back run. With overlapped launches (HDFS3_LAUNCH_OVERLAP_PREVIOUS) a
kernel's duration exceeds the interval at which launches complete; the interval is what
bench.py's HIP events over the timed region divide by K.

    python tools/trace_intervals.py gpurun_out/prof_bench/run_kernel_trace.csv [name-substring]
"""
import csv
import json
import statistics
import sys


def main():
    path = sys.argv[1]
    needle = sys.argv[2] if len(sys.argv) > 2 else "crc32c_wave_kernel<512, true"
    rows = [r for r in csv.DictReader(open(path)) if needle in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    # back-to-back runs (start-to-start gaps under 100 us), in launch order; bench.py's order
    # is: diagnostic pass (K, events between launches), warmup (W), TIMED region (K),
    # barriered warmup (W), barriered region (K)
    runs, cur = [], 0
    for i in range(1, len(st) + 1):
        if i == len(st) or st[i] - st[i - 1] > 100_000:
            if i - cur >= 100:
                runs.append((cur, i))
            cur = i
    for a, b in runs:
        dur = [(en[i] - st[i]) / 1e3 for i in range(a, b)]
        gaps = [(st[i + 1] - st[i]) / 1e3 for i in range(a, b - 1)]
        print(json.dumps({"kernel": needle, "dispatches": b - a, "avg_duration_us": round(statistics.mean(dur), 3),
                          "median_duration_us": round(statistics.median(dur), 3),
                          "avg_dispatch_interval_us": round(statistics.mean(gaps), 3),
                          "region_us_per_launch": round((en[b - 1] - st[a]) / 1e3 / (b - a), 3)}))


if __name__ == "__main__":
    main()
