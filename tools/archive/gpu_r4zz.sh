#!/bin/bash
# Round 4, last check of the committed tree: the full -m gpu suite and smoke().
set -o pipefail
TAG=${1:-r4zz}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 \
    && tail -1 gpurun_out/${TAG}_smoke.txt
