#!/bin/bash
# Chunks above 4 KiB through pieces + combine: the whole -m gpu suite, A/B against the multi-round
# kernel (lab 123) at 1 GiB per launch, both modes.
set -o pipefail
TAG=${1:-r3zf}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_gpu_tests.txt | head -30; exit $rc; }
ab() { # name args...
    local n=$1; shift
    timeout -k 10 200 python3 tools/ab.py "$@" > gpurun_out/${TAG}_$n.jsonl 2> gpurun_out/${TAG}_$n.err || { echo "ab $n failed"; tail -3 gpurun_out/${TAG}_$n.err; exit 1; }
    echo "== $n"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['bpc'], j['mode'], j['case'], j['us_med'], j['us_min'], j['results_ok'])" gpurun_out/${TAG}_$n.jsonl
}
ab big_bar --variants 0,123 --bpc 4096,8192,16384,65536 --block-mib 1024 --blocks 2 --reps 6 --rounds 5 || exit 1
ab big_ovl --variants 0,123 --bpc 8192,65536 --block-mib 1024 --blocks 2 --reps 6 --rounds 5 --overlap || exit 1
ab big_cmp --variants 0,123 --bpc 8192,65536 --block-mib 1024 --blocks 2 --reps 6 --rounds 5 --mode compute || exit 1
ab b128_bar --variants 0,123 --bpc 8192 --rounds 7 || exit 1
