#!/bin/bash
# Config 5 on the final round-3 build (tools/e2e_read.py) and the write path (tools/e2e_write.py).
set -o pipefail
TAG=${1:-r3e2e}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/e2e_read.py > gpurun_out/${TAG}_e2e_read.jsonl 2> gpurun_out/${TAG}_e2e_read.err \
    || { echo "e2e_read failed"; tail -20 gpurun_out/${TAG}_e2e_read.err; exit 1; }
cut -c1-220 gpurun_out/${TAG}_e2e_read.jsonl
timeout -k 10 300 python -u tools/e2e_write.py > gpurun_out/${TAG}_e2e_write.jsonl 2> gpurun_out/${TAG}_e2e_write.err \
    || { echo "e2e_write failed"; tail -20 gpurun_out/${TAG}_e2e_write.err; exit 1; }
cut -c1-220 gpurun_out/${TAG}_e2e_write.jsonl
