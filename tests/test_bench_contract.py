"""bench.py keeps the driver's JSON contract (one line on stdout, rank 0): the BASELINE.json
metric, a whole-job `value`, `roofline` for the dominant kernel and the barriered/batched
side measurements. A short run on the GPU box; the PMC passes and the CPU baseline are
skipped here (the round-end bench runs them)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(320)  # the verify line carries configs[2] and configs[4] too (~1 min on the box)
@pytest.mark.parametrize("mode", ["verify", "compute"])
def test_bench_json_line(mode):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "50", "--warmup", "10", "--no-pmc",
           "--no-cpu-baseline", "--mode", mode]
    out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    j = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in j, key
    assert j["n_gpus"] == 1 and j["steps"] == 50 and j["warmup"] == 10
    assert j["unit"] == "GiB/s" and j["value"] > 0 and j["higher_is_better"] is True
    assert j["scaling"] == "weak" and j["dtype"] == "u8"
    assert j["config"]["mode"] == mode and j["config"]["block_bytes"] == 128 << 20
    r = j["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] <= 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    # verify reads data + words; compute reads data and writes words: same algorithmic bytes
    assert r["alg_bytes_per_launch"] == 262144 * (512 + 4)
    # the untimed launches before the timed region are disclosed beside `warmup`
    pp = j["pre_pass_launches"]
    assert pp["warmup"] == 10 and pp["total_before_timed_region"] == sum(v for k, v in pp.items()
                                                                         if k != "total_before_timed_region")
    if mode != "verify":
        return
    # BASELINE.json configs[2]: 1 GiB per launch, compute + verify at bpc 512 / 2048 / 4096, both forms
    c2 = j["configs2"]
    assert c2["bytes_per_launch"] == 1 << 30 and sorted(c2["bpc"]) == ["2048", "4096", "512"]
    for bpc, row in c2["bpc"].items():
        assert row["alg_bytes_per_launch"] == (1 << 30) // int(bpc) * (int(bpc) + 4)
        for m in ("verify", "compute"):
            for form in ("overlapped", "barriered"):
                assert 0 < row[m][form]["frac"] <= 1, (bpc, m, form)
        assert 0.5 < row["compute_vs_verify"]["overlapped"] < 1.5 and "checked" in row
    # BASELINE.json configs[4]: loopback hdfsRead of 1 GiB, PCIe-inclusive, the reference CPU path beside it
    c5 = j["config5"]["lines"]
    for k in ("hdfsRead_verify", "hdfsRead_no_verify", "hdfsRead_verify_readahead2", "host_api_pinned",
              "host_api_pageable", "hdfsWrite_sink"):
        assert c5[k]["gib_s"] > 0 and len(c5[k]["gib_s_all"]) == 5, k
    if "reference_cpu_verify" in c5:  # oracle/_ref travels with the tree when it was built
        assert c5["reference_cpu_verify"]["kind"] == "reference" and c5["reference_cpu_verify"]["gib_s"] > 0
        assert c5["reference_cpu_write_sink"]["gib_s"] > 0 and "checked" in c5["hdfsWrite_sink"]
        pr = j["config5"]["paired_gpu_over_reference_cpu"]
        for k in ("verify", "no_verify", "verify_8_streams", "no_verify_8_streams"):
            assert pr[k]["rate"] > 0 and pr[k]["client_cpu"] > 0, k
        # round 6: 8 concurrent streams on both paths, CPU-seconds per GiB on every read line, the
        # datanode in its own process (its CPU apart), the reader's phases on the GPU lines
        for k in ("hdfsPread8_verify", "reference_cpu8_verify"):
            assert c5[k]["gib_s"] > 0 and c5[k]["streams"] == 8, k
        for k in ("hdfsRead_verify", "reference_cpu_verify", "hdfsPread8_verify", "reference_cpu8_verify"):
            assert c5[k]["client_cpu_s_per_gib"] > 0 and c5[k]["datanode_cpu_s_per_gib"] > 0, k
            assert "cgroup_throttled_s_per_s" in c5[k], k
        ph = c5["hdfsPread8_verify"]["reader_phase_s_per_gib"]
        assert ph["recv"] > 0 and ph["receiver_cpu"] > 0
        assert j["config5"]["datanode"].startswith("a child process")
    # round 6: the output stream's own 64-packet batch (127-chunk packets at bpc 512), device-resident
    wb = j["packets"]["writer_batch"]
    assert wb["chunks_per_packet"] == 127 and wb["packet_data_bytes"] == 65024 and wb["packets_per_batch"] == 64
    assert wb["compute_us"] > 0 and 0 < wb["compute_frac"] < 1 and wb["reader_dense_us"] > 0
