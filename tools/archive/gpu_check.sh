#!/bin/bash
# One GPU-box pass: the -m gpu suite, smoke(), the default bench line, and the kernel trace of
# the same bench command. Every GPU step has its own time limit; the first failure ends the call.
# Usage (gpurun): bash tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-check}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1 \
    || { echo "gpu tests failed"; tail -40 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 \
    || { echo "smoke failed"; cat gpurun_out/${TAG}_smoke.txt; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run \
    -- python3 bench.py --no-pmc --no-cpu-baseline > gpurun_out/${TAG}_bench_prof.json 2> gpurun_out/${TAG}_bench_prof.err \
    || { echo "profiled bench failed"; tail -20 gpurun_out/${TAG}_bench_prof.err; exit 1; }
cat gpurun_out/${TAG}_bench_prof.json
