#!/bin/bash
# Round 4 closing pass on the final build: the -m gpu suite, smoke(), the driver's bench command and
# the default one, a kernel trace + stats of the driver's command, PMC passes of the verify kernel
# (overlapped and barriered, one rocprofv3 pass per counter group) and the per-launch clock probe.
set -o pipefail
TAG=${1:-r4z}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.txt | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 \
    || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
summ() { python3 -c "import json; d=json.load(open('$1')); r=d['roofline']; print('$1', 'value', d['value'], 'us', r['avg_launch_us'], 'frac', r['frac'], 'same', r.get('frac_of_achievable_same_form'), 'ach', r.get('frac_of_achievable_per_block'), 'bar', d['barriered']['frac'], d['barriered'].get('frac_of_achievable_per_block'), 'pk', d['packets']['overlapped']['frac_vs_contiguous'], d['packets']['barriered']['frac_vs_contiguous'], 'cmp', d['compute']['overlapped']['frac_vs_verify'], d['compute']['overlapped']['paired']['compute_vs_verify'], d['compute']['barriered']['frac_vs_verify'], d['compute']['barriered']['paired']['compute_vs_verify'], 'batched', d['batched']['frac'], 'traffic', r.get('traffic'))"; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json \
    2> gpurun_out/${TAG}_bench_k20.err || { echo "bench k20 failed"; tail gpurun_out/${TAG}_bench_k20.err; exit 1; }
summ gpurun_out/${TAG}_bench_k20.json
timeout -k 10 300 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail gpurun_out/${TAG}_bench.err; exit 1; }
summ gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_k20tr -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline \
    > gpurun_out/${TAG}_k20tr.json 2> gpurun_out/${TAG}_k20tr.err || { echo "trace failed"; exit 1; }
f=$(ls gpurun_out/${TAG}_k20tr/run_kernel_trace.csv gpurun_out/${TAG}_k20tr/*/run_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 tools/trace_runs.py "$f" --min 5 > gpurun_out/${TAG}_k20tr_runs.txt && head -8 gpurun_out/${TAG}_k20tr_runs.txt
bash tools/pmc.sh gpurun_out/${TAG}_pmc_ovl --launches 16 --overlap || exit 1
bash tools/pmc.sh gpurun_out/${TAG}_pmc_bar --launches 16 || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_ovl > gpurun_out/${TAG}_pmc_ovl_summary.json
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_bar > gpurun_out/${TAG}_pmc_bar_summary.json
cat gpurun_out/${TAG}_pmc_ovl_summary.json
timeout -k 10 300 python -u tools/clock_ramp.py --reps 2 --kinds crc,compute,read --phases bench,steady \
    > gpurun_out/${TAG}_clock_ramp.jsonl 2> gpurun_out/${TAG}_clock_ramp.err; echo "clock rc=$?"
