#!/bin/bash
# Round counts skewed by slot quartile against the SIMD arbiter's oldest-first order (lab 126/127):
# coverage check, then in-process A/B at 128 MiB (overlapped, barriered). Both lost; the variants and
# its coverage check (tools/skew_check.py) exist only in commit 494a7a6 (removed after this run).
set -o pipefail
TAG=${1:-r3zj}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/skew_check.py > gpurun_out/${TAG}_check.txt 2>&1
rc=$?; echo "check rc=$rc"; tail -4 gpurun_out/${TAG}_check.txt; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift
  timeout -k 10 240 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run ovl --variants 0,126,127 --bpc 512 --rounds 9 --overlap &&
run bar --variants 0,126,127 --bpc 512 --rounds 9 &&
run ovl2 --variants 0,126,127 --bpc 512,4096 --rounds 9 --overlap &&
run bar2 --variants 0,126,127 --bpc 512,4096 --rounds 9
