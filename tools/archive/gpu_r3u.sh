#!/bin/bash
# Re-entry check of round 3 (rebuilt container): the -m gpu suite, smoke(), the kernel trace of the
# driver's bench command (K=20, W=5), and the A/B of the NCH-chain lab variants (crc32c_wave_n.h).
set -o pipefail
TAG=${1:-r3u}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 \
    || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
V=0,113,110,111,114,112
timeout -k 10 200 python3 tools/ab.py --variants $V --bpc 512 --rounds 7 --overlap > gpurun_out/${TAG}_ab_ovl.jsonl 2> gpurun_out/${TAG}_ab_ovl.err \
    || { echo "ab ovl failed"; tail -5 gpurun_out/${TAG}_ab_ovl.err; exit 1; }
timeout -k 10 200 python3 tools/ab.py --variants $V --bpc 512 --rounds 7 > gpurun_out/${TAG}_ab_bar.jsonl 2> gpurun_out/${TAG}_ab_bar.err \
    || { echo "ab bar failed"; tail -5 gpurun_out/${TAG}_ab_bar.err; exit 1; }
timeout -k 10 200 python3 tools/ab.py --variants $V --bpc 512 --rounds 5 --block-mib 1024 --blocks 2 --reps 6 > gpurun_out/${TAG}_ab_1g.jsonl 2> gpurun_out/${TAG}_ab_1g.err \
    || { echo "ab 1g failed"; tail -5 gpurun_out/${TAG}_ab_1g.err; exit 1; }
for f in ovl bar 1g; do echo "== $f"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l); print(j['case'], j['us_med'], j['us_min'], j['results_ok'])" gpurun_out/${TAG}_ab_$f.jsonl; done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_k20tr -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/${TAG}_k20tr.json 2> gpurun_out/${TAG}_k20tr.err \
    || { echo "k20 trace failed"; tail -20 gpurun_out/${TAG}_k20tr.err; exit 1; }
cat gpurun_out/${TAG}_k20tr.json
