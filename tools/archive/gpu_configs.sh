#!/bin/bash
# The BASELINE.json configs other than the bench line, on the current build: config 0 (one 64 KiB
# packet) and config 2 (1 GiB compute + verify, bpc 512/2048/4096) via tools/configs.py, config 5
# (PCIe-inclusive host verify, hdfsRead over the loopback datanode, short-circuit reads) via
# tools/e2e_read.py. Usage (gpurun): bash tools/gpu_configs.sh <tag>
set -o pipefail
TAG=${1:-cfg}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/configs.py > gpurun_out/${TAG}_configs.jsonl 2> gpurun_out/${TAG}_configs.err \
    || { echo "configs failed"; tail -20 gpurun_out/${TAG}_configs.err; exit 1; }
cat gpurun_out/${TAG}_configs.jsonl
timeout -k 10 500 python -u tools/e2e_read.py > gpurun_out/${TAG}_e2e_read.jsonl 2> gpurun_out/${TAG}_e2e_read.err \
    || { echo "e2e_read failed"; tail -20 gpurun_out/${TAG}_e2e_read.err; exit 1; }
cat gpurun_out/${TAG}_e2e_read.jsonl
