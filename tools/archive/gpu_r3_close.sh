#!/bin/bash
# Round-3 closing pass (re-entry session): the -m gpu suite, smoke(), the bench in the driver's form
# and the default form (PMC traffic included), the kernel trace of the default bench, PMC passes of
# the bench shape in both launch modes, the clock probe, and configs 0/2 (tools/configs.py).
set -o pipefail
TAG=${1:-r3c}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 \
    || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json 2> gpurun_out/${TAG}_bench_k20.err \
    || { echo "bench k20 failed"; tail -20 gpurun_out/${TAG}_bench_k20.err; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
for f in bench_k20 bench; do
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; b=j['barriered']; c=j['compute']; print(sys.argv[1], j['value'], r['avg_launch_us'], r['frac'], r.get('frac_of_achievable_per_block'), r.get('frac_of_achievable_same_form'), 'bar', b['frac'], b.get('frac_of_achievable_per_block'), 'batched', j['batched']['frac'], 'cmp', c['overlapped']['frac'], c['overlapped'].get('frac_vs_verify'), c['barriered']['frac'], c['barriered'].get('frac_vs_verify'), 'cpu', j['cpu_baseline']['value'], 'traffic', r.get('traffic'))" gpurun_out/${TAG}_$f.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
    python3 bench.py --steps 2000 --warmup 1000 --no-cpu-baseline --no-pmc \
    > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace_bench.err \
    || { echo "trace failed"; tail -20 gpurun_out/${TAG}_trace_bench.err; exit 1; }
python3 tools/trace_runs.py gpurun_out/${TAG}_trace/run_kernel_trace.csv > gpurun_out/${TAG}_trace_runs.txt || true
tail -4 gpurun_out/${TAG}_trace_runs.txt
bash tools/pmc.sh gpurun_out/${TAG}_pmc_ovl --launches 16 --overlap || exit 1
bash tools/pmc.sh gpurun_out/${TAG}_pmc_bar --launches 16 || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_ovl > gpurun_out/${TAG}_pmc_ovl_summary.json
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_bar > gpurun_out/${TAG}_pmc_bar_summary.json
python3 -c "import json; [print(f, json.load(open('gpurun_out/${TAG}_pmc_%s_summary.json' % f))['derived']) for f in ('ovl','bar')]"
timeout -k 10 120 python3 tools/clock_probe.py --seconds 3 --phases v0,readnt,v77 > gpurun_out/${TAG}_clk_ovl.jsonl 2>/dev/null || exit 1
python3 tools/clock_summary.py gpurun_out/${TAG}_clk_ovl.jsonl
timeout -k 10 300 python -u tools/configs.py > gpurun_out/${TAG}_configs.jsonl 2> gpurun_out/${TAG}_configs.err \
    || { echo "configs failed"; tail -20 gpurun_out/${TAG}_configs.err; exit 1; }
cat gpurun_out/${TAG}_configs.jsonl
