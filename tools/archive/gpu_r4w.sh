#!/bin/bash
# Round 4: the short-circuit reader's host-side knobs in child processes, and the pool-cap test.
set -o pipefail
TAG=${1:-r4w}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_local_reader.py -m gpu -q -k "knobs or pinned_cap" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || grep -E "^FAILED|^E " gpurun_out/${TAG}_tests.txt | head -20
