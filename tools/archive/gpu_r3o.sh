#!/bin/bash
# Round-3 pass: round kernel with 256 / 512 threads per workgroup (one workgroup per CU either way:
# 4 / 8 waves per CU instead of 16) against production; parity of the lab variants first.
set -o pipefail
TAG=${1:-r3o}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/${TAG}_parity.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab.py --variants 0,97,98 --bpc 512,2048,4096 --overlap --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_ovl.jsonl 2> gpurun_out/${TAG}_ab_ovl.err || { echo "ab failed"; tail gpurun_out/${TAG}_ab_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_ovl.jsonl
timeout -k 10 300 python -u tools/ab.py --variants 0,97,98 --bpc 512,4096 --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_bar.jsonl 2> gpurun_out/${TAG}_ab_bar.err || { echo "ab failed"; tail gpurun_out/${TAG}_ab_bar.err; exit 1; }
cat gpurun_out/${TAG}_ab_bar.jsonl
timeout -k 10 300 python -u tools/ab.py --variants 0,97,98 --bpc 512 --mode compute --overlap --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_cmp.jsonl 2> gpurun_out/${TAG}_ab_cmp.err || { echo "ab failed"; tail gpurun_out/${TAG}_ab_cmp.err; exit 1; }
cat gpurun_out/${TAG}_ab_cmp.jsonl
timeout -k 10 240 python -u tools/ab.py --variants 0,97,98 --bpc 512 --block-mib 1024 --blocks 2 --overlap --rounds 5 --reps 20 \
    > gpurun_out/${TAG}_ab_1g.jsonl 2> gpurun_out/${TAG}_ab_1g.err || { echo "ab 1g failed"; tail gpurun_out/${TAG}_ab_1g.err; exit 1; }
cat gpurun_out/${TAG}_ab_1g.jsonl
