#!/bin/bash
# Compute words staged in LDS at every size, written out window by window (lab 130), against
# production (staged up to bpc/16 rounds per wave, held / per-round stores beyond): parity, then
# in-process A/B at 1 GiB and 2 GiB, and 512 MiB (identical code below the limit).
set -o pipefail
TAG=${1:-r3zn}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.txt | head -30; exit $rc; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run c_1g --variants 0,130 --bpc 512,1024 --rounds 7 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap --mode compute &&
run c_1g_bar --variants 0,130 --bpc 512 --rounds 7 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --mode compute &&
run c_2g --variants 0,130 --bpc 512,2048 --rounds 5 --block-mib 2560 --blocks 2 --reps 4 --warm 100 --overlap --mode compute &&
run v_1g --variants 0 --bpc 512 --rounds 7 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap
