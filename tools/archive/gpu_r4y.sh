#!/bin/bash
# Round 4: uneven workgroups on overlapped launches (lab 153, kLabSkew) against production: parity,
# then 20-launch regions from an idle GPU (the driver's form) and 200-launch regions, 128 MiB.
set -o pipefail
TAG=${1:-r4y}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "variants_overlapped_match and 153" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/${TAG}_tests.txt | head; exit 1; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run k20 --variants 0,153 --rounds 15 --reps 20 --overlap &&
run k200 --variants 0,153 --rounds 7 --reps 200 --overlap &&
run k20b --variants 0,153 --rounds 15 --reps 20 --overlap
