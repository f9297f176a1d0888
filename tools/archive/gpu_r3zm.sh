#!/bin/bash
# Staged compute words at bpc 1024 / 2048 (kStageWords generalised): the parity tests that cover
# compute, then in-process A/B against per-round stores (lab 122) at 128 MiB and 1 GiB, and config 2.
set -o pipefail
TAG=${1:-r3zm}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_crc32.py -m gpu -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.txt | head -30; exit $rc; }
run() { local name=$1; shift
  timeout -k 10 240 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run c_ovl --variants 0,122 --bpc 1024,2048,512 --rounds 9 --overlap --mode compute &&
run c_bar --variants 0,122 --bpc 1024,2048,512 --rounds 9 --mode compute &&
run c_1g --variants 0,122 --bpc 1024,2048 --rounds 5 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap --mode compute &&
run v_1g --variants 0 --bpc 1024,2048 --rounds 5 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap &&
timeout -k 10 300 python -u tools/configs.py > gpurun_out/${TAG}_configs.jsonl 2> gpurun_out/${TAG}_configs.err
rc=$?; echo "configs rc=$rc"; grep config2 gpurun_out/${TAG}_configs.jsonl; exit $rc
