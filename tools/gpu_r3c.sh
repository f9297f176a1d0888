#!/bin/bash
# Round-3 pass: -m gpu suite, kernel A/B (late vs early prefetch, solo last step, round-2 kernel 90).
set -o pipefail
TAG=${1:-r3c}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
echo "gpu tests rc=$?"; tail -15 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 300 python -u tools/ab.py --variants 0,90,92,93,94 --bpc 512,4096 --overlap --rounds 9 --reps 100 \
    > gpurun_out/${TAG}_ab_ovl.jsonl 2> gpurun_out/${TAG}_ab_ovl.err || { echo "ab ovl failed"; tail gpurun_out/${TAG}_ab_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_ovl.jsonl
timeout -k 10 240 python -u tools/ab.py --variants 0,90,92 --bpc 512,4096 --rounds 9 --reps 100 \
    > gpurun_out/${TAG}_ab_bar.jsonl 2> gpurun_out/${TAG}_ab_bar.err || { echo "ab bar failed"; tail gpurun_out/${TAG}_ab_bar.err; exit 1; }
cat gpurun_out/${TAG}_ab_bar.jsonl
timeout -k 10 240 python -u tools/ab.py --mode compute --variants 0,90,92 --bpc 512,4096 --rounds 9 --reps 100 \
    > gpurun_out/${TAG}_ab_cmp.jsonl 2> gpurun_out/${TAG}_ab_cmp.err || { echo "ab cmp failed"; tail gpurun_out/${TAG}_ab_cmp.err; exit 1; }
cat gpurun_out/${TAG}_ab_cmp.jsonl
timeout -k 10 240 python -u tools/ab.py --variants 0,90,92 --bpc 512 --block-mib 1024 --blocks 2 --overlap --rounds 5 --reps 20 \
    > gpurun_out/${TAG}_ab_1g.jsonl 2> gpurun_out/${TAG}_ab_1g.err || { echo "ab 1g failed"; tail gpurun_out/${TAG}_ab_1g.err; exit 1; }
cat gpurun_out/${TAG}_ab_1g.jsonl
