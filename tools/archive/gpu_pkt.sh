#!/bin/bash
# GPU-box pass: full -m gpu suite, then the packet-stream rate tool.
set -o pipefail
TAG=${1:-pkt}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 300 python -u tools/packets_rate.py > gpurun_out/${TAG}_packets_rate.jsonl 2>&1 \
    || { echo "packets_rate failed"; tail -20 gpurun_out/${TAG}_packets_rate.jsonl; exit 1; }
cat gpurun_out/${TAG}_packets_rate.jsonl
timeout -k 10 400 python -u tools/e2e_write.py > gpurun_out/${TAG}_e2e_write.jsonl 2>&1 \
    || { echo "e2e_write failed"; tail -20 gpurun_out/${TAG}_e2e_write.jsonl; exit 1; }
cat gpurun_out/${TAG}_e2e_write.jsonl
