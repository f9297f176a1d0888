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
@pytest.mark.parametrize("mode", ["verify", "compute"])
def test_bench_json_line(mode):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "50", "--warmup", "10", "--no-pmc",
           "--no-cpu-baseline", "--mode", mode]
    out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=110)
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
