#!/bin/bash
# Write-path GPU tests (packets byte-identical to the reference model, pipelines, hdfs.h
# consumer), then the hdfsWrite rates. Usage (gpurun): bash tools/gpu_write.sh <tag>
set -o pipefail
TAG=${1:-write}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_output_stream.py tests/test_pipeline.py tests/test_abi_consumer.py \
    tests/test_block_checksum.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
timeout -k 10 400 python -u tools/e2e_write.py > gpurun_out/${TAG}_e2e_write.jsonl 2> gpurun_out/${TAG}_e2e_write.err \
    || { echo "e2e_write failed"; tail -20 gpurun_out/${TAG}_e2e_write.err; exit 1; }
cut -c1-220 gpurun_out/${TAG}_e2e_write.jsonl
