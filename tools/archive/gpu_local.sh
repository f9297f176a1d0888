#!/bin/bash
# short-circuit reader: GPU tests, then the local-read rates with mapped and pread staging
set -o pipefail
TAG=${1:-local}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_local_reader.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
timeout -k 10 400 python -u tools/e2e_read.py --local-only > gpurun_out/${TAG}_default.jsonl 2>&1 \
    || { echo "e2e default failed"; tail -20 gpurun_out/${TAG}_default.jsonl; exit 1; }
cat gpurun_out/${TAG}_default.jsonl
HDFS3_LOCAL_MMAP=1 timeout -k 10 400 python -u tools/e2e_read.py --local-only > gpurun_out/${TAG}_mmap1.jsonl 2>&1 \
    || { echo "e2e mmap1 failed"; tail -20 gpurun_out/${TAG}_mmap1.jsonl; exit 1; }
cat gpurun_out/${TAG}_mmap1.jsonl
