#!/bin/bash
# Round-3 pass: -m gpu suite, bench (batch pass: no event between barriered launches, its own
# warmup), config 5 with the read-ahead lines (pool cap in force), clock probe with the fixed
# no-math diagnostic.
set -o pipefail
TAG=${1:-r3k}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j[\"roofline\"]; print(\"k2000\", j[\"value\"], r[\"avg_launch_us\"], r[\"frac\"], r[\"frac_of_achievable_per_block\"], j[\"barriered\"][\"frac\"], j[\"barriered\"][\"frac_of_achievable_per_block\"], j[\"batched\"], j[\"compute\"][\"overlapped\"][\"frac_vs_verify\"], j[\"compute\"][\"barriered\"][\"frac_vs_verify\"])" gpurun_out/${TAG}_bench.json
timeout -k 10 500 python -u tools/e2e_read.py > gpurun_out/${TAG}_e2e_read.jsonl 2> gpurun_out/${TAG}_e2e_read.err \
    || { echo "e2e_read failed"; tail -20 gpurun_out/${TAG}_e2e_read.err; exit 1; }
cut -c1-220 gpurun_out/${TAG}_e2e_read.jsonl
P="v0,readnt,v77"
timeout -k 10 120 python3 tools/clock_probe.py --seconds 3 --phases $P > gpurun_out/${TAG}_clk_ovl.jsonl 2>/dev/null || exit 1
python3 tools/clock_summary.py gpurun_out/${TAG}_clk_ovl.jsonl
