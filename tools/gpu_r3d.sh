#!/bin/bash
# Round-3 pass: -m gpu suite on the production choice (late prefetch, solo last step overlapped,
# segment walk), then A/B: verify/compute overlapped, barriered, segments; then the bench line.
set -o pipefail
TAG=${1:-r3d}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
echo "gpu tests rc=$?"; tail -15 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 300 python -u tools/ab.py --variants 0,90,93,96 --bpc 512,4096 --overlap --rounds 11 --reps 100 \
    > gpurun_out/${TAG}_ab_ovl.jsonl 2> gpurun_out/${TAG}_ab_ovl.err || { echo "ab ovl failed"; tail gpurun_out/${TAG}_ab_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_ovl.jsonl
timeout -k 10 240 python -u tools/ab.py --mode compute --variants 0,90,93 --bpc 512 --overlap --rounds 11 --reps 100 \
    > gpurun_out/${TAG}_ab_cmp_ovl.jsonl 2> gpurun_out/${TAG}_ab_cmp_ovl.err || { echo "ab cmp failed"; tail gpurun_out/${TAG}_ab_cmp_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_cmp_ovl.jsonl
timeout -k 10 240 python -u tools/seg_ab.py > gpurun_out/${TAG}_seg_ab.jsonl 2> gpurun_out/${TAG}_seg_ab.err \
    || { echo "seg ab failed"; tail gpurun_out/${TAG}_seg_ab.err; exit 1; }
cat gpurun_out/${TAG}_seg_ab.jsonl
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
