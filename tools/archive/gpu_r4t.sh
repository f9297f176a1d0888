#!/bin/bash
# Round 4: rounds 2, 3 prefetched in the prologue (lab 151, kLabHeadPf) against production: parity,
# barriered / overlapped A/B (verify bpc 512 / 2048, compute 512; 4 MiB .. 1 GiB), per-wave head (152).
set -o pipefail
TAG=${1:-r4t}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "variants_overlapped and 151" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/${TAG}_tests.txt | head; exit 1; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run bar128 --variants 0,151 --bpc 512,2048 --rounds 7 --reps 100 &&
run ovl128 --variants 0,151 --bpc 512,2048 --rounds 7 --reps 100 --overlap &&
run cbar128 --variants 0,151 --mode compute --rounds 7 --reps 100 &&
run covl128 --variants 0,151 --mode compute --rounds 7 --reps 100 --overlap &&
run bar1g --variants 0,151 --rounds 5 --block-mib 1024 --blocks 2 --reps 20 &&
run bar32 --variants 0,151 --rounds 5 --block-mib 32 --blocks 16 --reps 100 &&
run bar4 --variants 0,151 --rounds 5 --block-mib 4 --blocks 128 --reps 100 || exit 1
timeout -k 10 300 python -u tools/wave_spread.py --k 40 --kinds crc --variant 152 --mid > gpurun_out/${TAG}_spread152.jsonl \
    2> gpurun_out/${TAG}_spread152.err; cat gpurun_out/${TAG}_spread152.jsonl
