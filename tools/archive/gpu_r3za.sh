#!/bin/bash
# The whole -m gpu suite on the prologue changes (host-split round counts, xor-permuted fill, no slow
# region for whole-round launches); where compute loses against verify at 128 MiB (held words not
# stored: 118, stored over one small region: 119); wave priority in the multi-round kernel (bpc >
# 4096, lab 117 = off); PMC passes of the bench shape.
set -o pipefail
TAG=${1:-r3za}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit $rc; }
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
ab r8k_bar --variants 0,117 --bpc 8192,65536 --block-mib 1024 --blocks 2 --reps 6 --rounds 7 || exit 1
ab r8k_ovl --variants 0,117 --bpc 8192 --block-mib 1024 --blocks 2 --reps 6 --rounds 7 --overlap || exit 1
bash tools/pmc.sh gpurun_out/${TAG}_pmc_ovl --launches 16 --overlap || exit 1
bash tools/pmc.sh gpurun_out/${TAG}_pmc_bar --launches 16 || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_ovl > gpurun_out/${TAG}_pmc_ovl_summary.json
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_bar > gpurun_out/${TAG}_pmc_bar_summary.json
python3 -c "import json; [print(f, json.load(open('gpurun_out/${TAG}_pmc_%s_summary.json' % f))['derived']) for f in ('ovl','bar')]"
