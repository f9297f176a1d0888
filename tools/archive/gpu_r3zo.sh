#!/bin/bash
# Windowed staging in production at bpc 1024 / 2048 (past 1 GiB / 2 GiB per launch): the -m gpu suite,
# smoke(), then A/B against per-round stores (lab 122) past the window size, bpc 512 held stores
# against windows (lab 130) at 1 GiB, and 128 MiB compute unchanged.
set -o pipefail
TAG=${1:-r3zo}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 \
    || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run c_big --variants 0,122 --bpc 1024,2048 --rounds 5 --block-mib 2560 --blocks 2 --reps 4 --warm 100 --overlap --mode compute &&
run c_1g --variants 0,130 --bpc 512 --rounds 5 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap --mode compute &&
run c_128 --variants 0,122 --bpc 512,1024,2048 --rounds 7 --overlap --mode compute &&
run v_big --variants 0 --bpc 1024,2048 --rounds 5 --block-mib 2560 --blocks 2 --reps 4 --warm 100 --overlap
