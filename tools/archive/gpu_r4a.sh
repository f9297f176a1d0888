#!/bin/bash
# Round-4 first pass on the round-3 final build: the -m gpu suite, smoke(), the driver's bench
# command and the default one, and a kernel trace of the driver's command (per-dispatch durations
# of the timed region, tools/trace_runs.py).
set -o pipefail
TAG=${1:-r4a}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
# assertion failures (rc 1) are reported and the measurements still run; a crash, abort or time
# limit ends the call here
[ $rc -eq 0 ] || grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.txt | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 \
    || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json \
    2> gpurun_out/${TAG}_bench_k20.err || { echo "bench k20 failed"; tail gpurun_out/${TAG}_bench_k20.err; exit 1; }
cat gpurun_out/${TAG}_bench_k20.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_k20tr -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline \
    > gpurun_out/${TAG}_k20tr.json 2> gpurun_out/${TAG}_k20tr.err || { echo "trace failed"; exit 1; }
f=$(ls gpurun_out/${TAG}_k20tr/*/run_kernel_trace.csv gpurun_out/${TAG}_k20tr/run_kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 tools/trace_runs.py "$f" --min 5 > gpurun_out/${TAG}_k20tr_runs.txt
cat gpurun_out/${TAG}_k20tr_runs.txt
