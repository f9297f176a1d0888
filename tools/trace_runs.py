#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace (run_kernel_trace.csv) into runs of consecutive dispatches of the
same kernel instantiation and print, per run: count, average duration, start-to-start interval,
idle between one dispatch's end and the next one's start, and the first/last durations.

    python3 tools/trace_runs.py gpurun_out/<dir>/run_kernel_trace.csv [--min 5]
"""
import csv
import re
import sys


def short(name):
    m = re.search(r"(crc32c_\w+|stream_read_kernel)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    return name.split("(")[0][-40:]


def main():
    path = sys.argv[1]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs = []
    for r in rows:
        k = short(r["Kernel_Name"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if runs and runs[-1][0] == k:
            runs[-1][1].append((s, e))
        else:
            runs.append([k, [(s, e)]])
    for k, ts in runs:
        if len(ts) < mn:
            continue
        d = [(e - s) / 1e3 for s, e in ts]
        st = [(ts[i + 1][0] - ts[i][0]) / 1e3 for i in range(len(ts) - 1)]
        idle = [max(0.0, (ts[i + 1][0] - ts[i][1]) / 1e3) for i in range(len(ts) - 1)]
        avg = lambda v: sum(v) / len(v) if v else 0.0
        print(f"{k:60s} n={len(ts):5d} dur={avg(d):7.2f} start2start={avg(st):7.2f} idle={avg(idle):6.2f} "
              f"first={[round(x, 1) for x in d[:4]]} last={[round(x, 1) for x in d[-3:]]}")


if __name__ == "__main__":
    main()
