#!/bin/bash
# Round-3 pass on the cleaned-up kernel set: the -m gpu suite, A/B of production (0: late prefetch,
# solo last step outside the loop) against early prefetch (92) and no solo (93), then the bench line.
set -o pipefail
TAG=${1:-r3h}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tests.txt
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u tools/ab.py --variants 0,92,93 --bpc 512,2048,4096 --overlap --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_ovl.jsonl 2> gpurun_out/${TAG}_ab_ovl.err || { echo "ab ovl failed"; tail gpurun_out/${TAG}_ab_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_ovl.jsonl
timeout -k 10 300 python -u tools/ab.py --variants 0,92 --bpc 512,4096 --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_bar.jsonl 2> gpurun_out/${TAG}_ab_bar.err || { echo "ab bar failed"; tail gpurun_out/${TAG}_ab_bar.err; exit 1; }
cat gpurun_out/${TAG}_ab_bar.jsonl
timeout -k 10 300 python -u tools/ab.py --variants 0,92 --bpc 512 --mode compute --overlap --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_cmp.jsonl 2> gpurun_out/${TAG}_ab_cmp.err || { echo "ab cmp failed"; tail gpurun_out/${TAG}_ab_cmp.err; exit 1; }
cat gpurun_out/${TAG}_ab_cmp.jsonl
timeout -k 10 240 python -u tools/ab.py --variants 0,93 --bpc 512 --block-mib 1024 --blocks 2 --overlap --rounds 5 --reps 20 \
    > gpurun_out/${TAG}_ab_1g.jsonl 2> gpurun_out/${TAG}_ab_1g.err || { echo "ab 1g failed"; tail gpurun_out/${TAG}_ab_1g.err; exit 1; }
cat gpurun_out/${TAG}_ab_1g.jsonl
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
