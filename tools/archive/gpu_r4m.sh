#!/bin/bash
# Round 4: rounds claimed from the workgroup's pool (lab 138, DynWalk): parity over the variant test
# (overlapped chains, 1-9 rounds per wave, bad chunks located), then in-process A/B against production
# barriered and overlapped at 128 MiB, 1 GiB, 32 MiB, bpc 512 and 2048, and the per-wave spread.
set -o pipefail
TAG=${1:-r4m}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "variants_overlapped_match" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/${TAG}_tests.txt | head; exit 1; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run bar128 --variants 0,138 --bpc 512,2048 --rounds 7 --reps 100 &&
run ovl128 --variants 0,138 --bpc 512,2048 --rounds 7 --reps 100 --overlap &&
run bar1g --variants 0,138 --rounds 5 --block-mib 1024 --blocks 2 --reps 20 &&
run ovl1g --variants 0,138 --rounds 5 --block-mib 1024 --blocks 2 --reps 20 --overlap &&
run bar32 --variants 0,138 --rounds 5 --block-mib 32 --blocks 16 --reps 100 || exit 1
timeout -k 10 300 python -u tools/wave_spread.py --k 40 --kinds crc --variant 139 > gpurun_out/${TAG}_spread139.jsonl \
    2> gpurun_out/${TAG}_spread139.err && cat gpurun_out/${TAG}_spread139.jsonl
