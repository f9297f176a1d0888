#!/bin/bash
# Round-3 profiles: kernel trace + stats of the bench command, the PMC passes of the verify
# kernel (overlapped and barriered, one rocprofv3 pass per counter group), the clock/power probe.
set -o pipefail
TAG=${1:-r3prof}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
    python3 bench.py --steps 2000 --warmup 1000 --no-cpu-baseline --no-pmc --no-compute \
    > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.err \
    || { echo "trace failed"; tail -20 gpurun_out/${TAG}_trace_bench.err; exit 1; }
cat gpurun_out/${TAG}_trace_bench.json
bash tools/pmc.sh gpurun_out/${TAG}_pmc_ovl --launches 16 --overlap || exit 1
bash tools/pmc.sh gpurun_out/${TAG}_pmc_bar --launches 16 || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_ovl > gpurun_out/${TAG}_pmc_ovl_summary.json
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_bar > gpurun_out/${TAG}_pmc_bar_summary.json
cat gpurun_out/${TAG}_pmc_ovl_summary.json gpurun_out/${TAG}_pmc_bar_summary.json
P="v0,readnt,v77"
timeout -k 10 120 python3 tools/clock_probe.py --seconds 3 --phases $P > gpurun_out/${TAG}_clk_ovl.jsonl 2>/dev/null || exit 1
timeout -k 10 120 python3 tools/clock_probe.py --seconds 3 --phases $P --barriered > gpurun_out/${TAG}_clk_bar.jsonl 2>/dev/null || exit 1
for f in ovl bar; do echo "== $f"; python3 tools/clock_summary.py gpurun_out/${TAG}_clk_$f.jsonl; done
