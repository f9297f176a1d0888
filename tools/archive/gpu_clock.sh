#!/bin/bash
# Power-limit study: sustained vs duty-cycled 128 MiB launches, overlapped and
# barriered, with amd-smi samples. Usage (gpurun): bash tools/gpu_clock.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P="v0,readnt,v77"
timeout -k 10 120 python3 tools/clock_probe.py --seconds 3 --phases $P > gpurun_out/clk_sustained_ovl.jsonl 2>/dev/null || exit 1
timeout -k 10 120 python3 tools/clock_probe.py --seconds 3 --phases $P --barriered > gpurun_out/clk_sustained_bar.jsonl 2>/dev/null || exit 1
timeout -k 10 120 python3 tools/clock_probe.py --seconds 3 --phases $P --burst 20 --gap-ms 4 > gpurun_out/clk_duty_ovl.jsonl 2>/dev/null || exit 1
timeout -k 10 120 python3 tools/clock_probe.py --seconds 3 --phases $P --burst 20 --gap-ms 4 --barriered > gpurun_out/clk_duty_bar.jsonl 2>/dev/null || exit 1
for f in sustained_ovl sustained_bar duty_ovl duty_bar; do echo "== $f"; python3 tools/clock_summary.py gpurun_out/clk_$f.jsonl; done
