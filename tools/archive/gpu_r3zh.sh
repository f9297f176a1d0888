#!/bin/bash
# Lane-mapping A/B: production (16 permlane swaps per round) against one permlane stage (124) and
# direct 64-byte lane loads (125), 128 MiB per launch overlapped / barriered, compute, and 1 GiB.
# Both lost (+16 % / +72 %); the variants exist only in commit 51b6ce7 (reverted after this run).
set -o pipefail
TAG=${1:-r3zh}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -k 10 240 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run ovl --variants 0,124,125 --bpc 512 --rounds 9 --overlap &&
run bar --variants 0,124,125 --bpc 512 --rounds 9 &&
run cmp --variants 0,124,125 --bpc 512 --rounds 7 --overlap --mode compute &&
run b2k --variants 0,124,125 --bpc 2048,4096 --rounds 5 --overlap &&
run 1g --variants 0,124,125 --bpc 512 --rounds 5 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap
