#!/bin/bash
# Reader/host-API GPU tests, then config 5 (tools/e2e_read.py, with the read-ahead lines).
# Usage (gpurun): bash tools/gpu_e2e.sh <tag>
set -o pipefail
TAG=${1:-e2e}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_input_readahead.py tests/test_input_stream.py tests/test_block_reader.py \
    tests/test_block_reader_malformed.py tests/test_local_reader.py tests/test_abi_consumer.py tests/test_gpu_parity.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
timeout -k 10 500 python -u tools/e2e_read.py > gpurun_out/${TAG}_e2e_read.jsonl 2> gpurun_out/${TAG}_e2e_read.err \
    || { echo "e2e_read failed"; tail -20 gpurun_out/${TAG}_e2e_read.err; exit 1; }
cut -c40-200 gpurun_out/${TAG}_e2e_read.jsonl
