#!/bin/bash
# Prefetch issue point A/B: production (before the chains) against after the chains' 4th / 8th word
# (lab 128 / 129: fewer bytes in flight per wave), 128 MiB overlapped / barriered, bpc 512 / 4096, 1 GiB.
# Within noise of production; the variants exist only in commit 0e81d7e (removed after this run).
set -o pipefail
TAG=${1:-r3zk}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -k 10 240 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run ovl --variants 0,128,129 --bpc 512,4096 --rounds 9 --overlap &&
run bar --variants 0,128,129 --bpc 512,4096 --rounds 9 &&
run cmp --variants 0,128,129 --bpc 512 --rounds 7 --overlap --mode compute &&
run 1g --variants 0,128,129 --bpc 512 --rounds 5 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap
