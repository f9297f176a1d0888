#!/bin/bash
# Round-3 pass: -m gpu suite, prefetch-timing A/B (mixed late/early per step pair), compute overlapped.
set -o pipefail
TAG=${1:-r3e}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
echo "gpu tests rc=$?"; tail -4 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 300 python -u tools/ab.py --variants 0,90,97,98 --bpc 512,4096 --overlap --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_ovl.jsonl 2> gpurun_out/${TAG}_ab_ovl.err || { echo "ab ovl failed"; tail gpurun_out/${TAG}_ab_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_ovl.jsonl
timeout -k 10 300 python -u tools/ab.py --variants 0,90,97,98 --bpc 512 --rounds 11 --reps 100 \
    > gpurun_out/${TAG}_ab_bar.jsonl 2> gpurun_out/${TAG}_ab_bar.err || { echo "ab bar failed"; tail gpurun_out/${TAG}_ab_bar.err; exit 1; }
cat gpurun_out/${TAG}_ab_bar.jsonl
timeout -k 10 240 python -u tools/ab.py --mode compute --variants 0,90,97,98 --bpc 512 --overlap --rounds 11 --reps 100 \
    > gpurun_out/${TAG}_ab_cmp_ovl.jsonl 2> gpurun_out/${TAG}_ab_cmp_ovl.err || { echo "ab cmp failed"; tail gpurun_out/${TAG}_ab_cmp_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_cmp_ovl.jsonl
