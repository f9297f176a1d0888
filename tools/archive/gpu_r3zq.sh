#!/bin/bash
# Compute at bpc 4096: 64 rounds' words held in one VGPR (lab 131) against per-round stores:
# the variant parity test, then in-process A/B at 128 MiB and 1 GiB.
set -o pipefail
TAG=${1:-r3zq}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "every_kernel_variant" --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.txt | head -30; exit $rc; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run c_128 --variants 0,131 --bpc 4096 --rounds 9 --overlap --mode compute &&
run c_128b --variants 0,131 --bpc 4096 --rounds 9 --mode compute &&
run c_1g --variants 0,131 --bpc 4096 --rounds 7 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap --mode compute &&
run v_1g --variants 0 --bpc 4096 --rounds 7 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap
