#!/bin/bash
# Round 4: a workgroup's waves one grid apart (lab 143, kLabSpread) against production, and whether
# the late CUs of a barriered 128 MiB launch are the same ones every launch (wave_spread, 125 / 144).
set -o pipefail
TAG=${1:-r4o}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "variants_overlapped_match and (143 or -0-)" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/${TAG}_tests.txt | head; exit 1; }
timeout -k 10 300 python -u tools/wave_spread.py --k 40 --kinds crc --variant 125 > gpurun_out/${TAG}_spread125.jsonl \
    2> gpurun_out/${TAG}_spread125.err && cat gpurun_out/${TAG}_spread125.jsonl || exit 1
timeout -k 10 300 python -u tools/wave_spread.py --k 40 --kinds crc --variant 144 > gpurun_out/${TAG}_spread144.jsonl \
    2> gpurun_out/${TAG}_spread144.err && cat gpurun_out/${TAG}_spread144.jsonl || exit 1
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run bar128 --variants 0,143 --bpc 512,2048 --rounds 7 --reps 100 &&
run ovl128 --variants 0,143 --bpc 512,2048 --rounds 7 --reps 100 --overlap &&
run bar1g --variants 0,143 --rounds 5 --block-mib 1024 --blocks 2 --reps 20 &&
run ovl1g --variants 0,143 --rounds 5 --block-mib 1024 --blocks 2 --reps 20 --overlap &&
run bar32 --variants 0,143 --rounds 5 --block-mib 32 --blocks 16 --reps 100
