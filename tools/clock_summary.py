#!/usr/bin/env python3
"""Summarise tools/clock_probe.py output: per phase, the median per-launch time of its
batches and the SMI samples taken while it ran (gfx clock range, socket power, UMC/GFX
activity, package-power-tracking throttle). One JSON line per phase.

    python tools/clock_summary.py gpurun_out/clock_probe.jsonl
"""
import json
import statistics
import sys


def main():
    rows = [json.loads(ln) for ln in open(sys.argv[1]) if ln.strip()]
    batches = [r for r in rows if "phase" in r]
    samples = [r["sample"] for r in rows if "sample" in r and isinstance(r["sample"].get("smi"), dict)]
    phases = []
    for r in batches:
        if not phases or phases[-1]["k"] != r.get("k", r["phase"]):
            phases.append({"k": r.get("k", r["phase"]), "phase": r["phase"], "t0": r["t"], "t1": r["t"], "us": []})
        phases[-1]["t1"] = r["t"]
        phases[-1]["us"].append(r["us_per_launch"])
    for p in phases:
        # samples wholly inside the phase, skipping its first 0.5 s (clock and power settle)
        inside = [s for s in samples if s["t"] >= p["t0"] + 0.5 and s["t_end"] <= p["t1"]]
        clk, pw, umc, gfx, ppt = [], [], [], [], []
        for s in inside:
            d = s["smi"]["gpu_data"][0]
            clk += [d["clock"][k]["clk"]["value"] for k in d["clock"] if k.startswith("gfx_")]
            pw.append(d["power"]["socket_power"]["value"])
            umc.append(d["usage"]["umc_activity"]["value"])
            gfx.append(d["usage"]["gfx_activity"]["value"])
            t = d.get("throttle", {})
            if isinstance(t.get("ppt_violation_activity"), dict):
                ppt.append(t["ppt_violation_activity"]["value"])
        print(json.dumps({
            "phase": p["phase"], "batches": len(p["us"]),
            "us_per_launch_median": round(statistics.median(p["us"]), 3),
            "us_per_launch_last10": round(statistics.mean(p["us"][-10:]), 3),
            "samples": len(inside),
            "gfx_clk_mhz": [min(clk), round(statistics.mean(clk)), max(clk)] if clk else None,
            "socket_power_w": round(statistics.mean(pw)) if pw else None,
            "umc_activity_pct": round(statistics.mean(umc)) if umc else None,
            "gfx_activity_pct": round(statistics.mean(gfx)) if gfx else None,
            "ppt_violation_activity_pct": round(statistics.mean(ppt)) if ppt else None,
        }))


if __name__ == "__main__":
    main()
