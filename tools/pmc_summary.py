#!/usr/bin/env python3
"""Per-dispatch averages of the counters collected by tools/pmc.sh for one kernel (default: the
512 B verify wave kernel), plus the derived per-round figures docs/DESIGN_HISTORY.md §5 quotes.

    python tools/pmc_summary.py <pmc_out_dir> [kernel-name-substring] [rounds_per_wave]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out = sys.argv[1]
    needle = sys.argv[2] if len(sys.argv) > 2 else "crc32c_wave_kernel<512, true"
    rounds_per_wave = float(sys.argv[3]) if len(sys.argv) > 3 else 8.0  # 128 MiB / 4096 waves / 4 KiB
    tot, disp = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if needle not in r.get("Kernel_Name", ""):
                continue
            name = r["Counter_Name"]
            tot[name] += float(r["Counter_Value"])
            disp[name].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    avg = {k: round(v / max(1, len(disp[k])), 1) for k, v in sorted(tot.items())}
    n = max((len(d) for d in disp.values()), default=0)
    waves = avg.get("SQ_WAVES", 4096.0)
    rounds = waves * rounds_per_wave
    derived = {}
    if "SQ_INSTS_LDS" in avg:
        derived["SQ_INSTS_LDS_per_round_per_wave"] = round(avg["SQ_INSTS_LDS"] / rounds, 2)
    if "SQ_INSTS_VALU" in avg:
        derived["SQ_INSTS_VALU_per_round"] = round(avg["SQ_INSTS_VALU"] / rounds, 1)
    if "SQ_LDS_BANK_CONFLICT" in avg:
        derived["lds_bank_conflict_cycles_per_launch"] = avg["SQ_LDS_BANK_CONFLICT"]
    if "FETCH_SIZE" in avg:
        # FETCH_SIZE in KiB, doubled on gfx950 (MI355X_MICROARCH.md, HBM/rocprofv3 section)
        derived["dram_bytes_per_launch"] = round(avg["FETCH_SIZE"] * 2 * 1024 + avg.get("WRITE_SIZE", 0) * 1024)
    print(json.dumps({**avg, "n_dispatches": n, "kernel": needle, "derived": derived}, indent=1))


if __name__ == "__main__":
    main()
