#!/bin/bash
# Where compute-on-write loses against verify at 128 MiB: held words not stored (118) or stored over
# one small region (119), in both launch modes, against production compute and production verify.
set -o pipefail
TAG=${1:-r3za}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ab() { # name args...
    local n=$1; shift
    timeout -k 10 200 python3 tools/ab.py "$@" > gpurun_out/${TAG}_$n.jsonl 2> gpurun_out/${TAG}_$n.err || { echo "ab $n failed"; tail -3 gpurun_out/${TAG}_$n.err; exit 1; }
    echo "== $n"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['bpc'], j['mode'], j['case'], j['us_med'], j['us_min'], j['results_ok'])" gpurun_out/${TAG}_$n.jsonl
}
ab c128_ovl --variants 0,118,119 --mode compute --rounds 9 --overlap || exit 1
ab v128_ovl --variants 0 --rounds 9 --overlap || exit 1
ab c128_bar --variants 0,118,119 --mode compute --rounds 9 || exit 1
ab v128_bar --variants 0 --rounds 9 || exit 1
