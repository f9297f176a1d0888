#!/bin/bash
# Round 4: compute-on-write overlapped against verify (the staged words' store policy: lab 126-128;
# held stores 122; no stores 118), the packet stream's solo step against the old path on one box,
# and config 5 (tools/e2e_read.py: read-ahead rings sized to the pinned cap).
set -o pipefail
TAG=${1:-r4e}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "variants_overlapped_compute" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.txt | head; exit $rc; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run cmp_ovl --variants 0,122,126,127,128,118 --rounds 7 --overlap --mode compute &&
run ver_ovl --variants 0 --rounds 7 --overlap --mode verify &&
run cmp_bar --variants 0,126,127 --rounds 5 --mode compute || exit 1
timeout -k 10 300 python -u tools/pkt_ab.py --variants 0,124 --rounds 7 --overlap > gpurun_out/${TAG}_pkt_ab.jsonl \
    2> gpurun_out/${TAG}_pkt_ab.err && cat gpurun_out/${TAG}_pkt_ab.jsonl || exit 1
timeout -k 10 600 python -u tools/e2e_read.py --readahead 1,3,7 --reps 3 > gpurun_out/${TAG}_e2e_read.jsonl \
    2> gpurun_out/${TAG}_e2e_read.err; rc=$?; echo "e2e rc=$rc"; cat gpurun_out/${TAG}_e2e_read.jsonl; exit $rc
