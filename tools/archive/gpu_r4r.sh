#!/bin/bash
# Round 4: is the 128 MiB launch's head the table images' loads? Diagnostic 148 makes the tables up
# (no loads; wrong results) against production, barriered and overlapped, and its per-wave
# fill-done / first-data times (147).
set -o pipefail
TAG=${1:-r4r}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run bar128 --variants 0,148 --rounds 7 --reps 100 &&
run ovl128 --variants 0,148 --rounds 7 --reps 100 --overlap &&
run bar4 --variants 0,148 --rounds 5 --block-mib 4 --blocks 128 --reps 100 || exit 1
timeout -k 10 300 python -u tools/wave_spread.py --k 40 --kinds crc --variant 147 --mid > gpurun_out/${TAG}_spread147.jsonl \
    2> gpurun_out/${TAG}_spread147.err; cat gpurun_out/${TAG}_spread147.jsonl
