#!/bin/bash
# Round 4: the solo last step on barriered launches (lab 145) against production (interleaved last
# step when barriered): parity (verify and compute variant tests), then barriered A/B at 4 MiB,
# 32 MiB, 128 MiB (verify bpc 512 / 2048, compute 512) and 1 GiB.
set -o pipefail
TAG=${1:-r4p}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "variants_overlapped and (145 or -0-)" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/${TAG}_tests.txt | head; exit 1; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run bar128 --variants 0,145 --bpc 512,2048 --rounds 7 --reps 100 &&
run cbar128 --variants 0,145 --mode compute --rounds 7 --reps 100 &&
run bar1g --variants 0,145 --rounds 5 --block-mib 1024 --blocks 2 --reps 20 &&
run bar32 --variants 0,145 --rounds 5 --block-mib 32 --blocks 16 --reps 100 &&
run bar4 --variants 0,145 --rounds 5 --block-mib 4 --blocks 128 --reps 100
