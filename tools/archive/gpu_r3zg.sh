#!/bin/bash
# Pieces threshold: the parity tests that cover chunks above 4 KiB.
set -o pipefail
TAG=${1:-r3zg}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_crc32.py -m gpu -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.txt | head -30; exit $rc; }
