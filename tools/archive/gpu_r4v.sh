#!/bin/bash
# Round 4: the short-circuit readers' pool under the pinned cap: local reader and read-ahead tests.
set -o pipefail
TAG=${1:-r4v}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_local_reader.py tests/test_input_readahead.py tests/test_abi.py -m gpu -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || grep -E "^FAILED|^E " gpurun_out/${TAG}_tests.txt | head -20
