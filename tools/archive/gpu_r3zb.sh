#!/bin/bash
# Compute at 128 MiB: the workgroup's waves meet at a barrier before their last flush (lab 120); words staged in LDS and written as whole lines (lab 121).
set -o pipefail
TAG=${1:-r3zb}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider -k "variant" > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/${TAG}_parity.txt
[ $rc -eq 0 ] || exit $rc
ab() { # name args...
    local n=$1; shift
    timeout -k 10 200 python3 tools/ab.py "$@" > gpurun_out/${TAG}_$n.jsonl 2> gpurun_out/${TAG}_$n.err || { echo "ab $n failed"; tail -3 gpurun_out/${TAG}_$n.err; exit 1; }
    echo "== $n"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['bpc'], j['mode'], j['case'], j['us_med'], j['us_min'], j['results_ok'])" gpurun_out/${TAG}_$n.jsonl
}
ab c128_ovl --variants 0,120,121,118 --mode compute --rounds 9 --overlap || exit 1
ab c128_bar --variants 0,120,121 --mode compute --rounds 9 || exit 1
ab c1g_ovl --variants 0,120 --mode compute --block-mib 1024 --blocks 2 --reps 6 --rounds 7 --overlap || exit 1
ab v128_ovl --variants 0 --rounds 9 --overlap || exit 1
