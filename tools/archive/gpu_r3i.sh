#!/bin/bash
# Round-3 pass: parity of the lab variants, then compute-mode A/B for overlapped launches:
# production (0: held stores, interleaved last step), solo last step (94), no held stores (95),
# both (96); verify A/B of 0 vs 93 once more.
set -o pipefail
TAG=${1:-r3i}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_crc32.py -m gpu -q --timeout 150 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_parity.txt 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/${TAG}_parity.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab.py --variants 0,94,95,96 --bpc 512 --mode compute --overlap --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_cmp_ovl.jsonl 2> gpurun_out/${TAG}_ab_cmp_ovl.err || { echo "ab failed"; tail gpurun_out/${TAG}_ab_cmp_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_cmp_ovl.jsonl
timeout -k 10 300 python -u tools/ab.py --variants 0,95 --bpc 512 --mode compute --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_cmp_bar.jsonl 2> gpurun_out/${TAG}_ab_cmp_bar.err || { echo "ab failed"; tail gpurun_out/${TAG}_ab_cmp_bar.err; exit 1; }
cat gpurun_out/${TAG}_ab_cmp_bar.jsonl
timeout -k 10 300 python -u tools/ab.py --variants 0,94,95,96 --bpc 512 --mode compute --block-mib 1024 --blocks 2 --overlap --rounds 5 --reps 20 \
    > gpurun_out/${TAG}_ab_cmp_1g.jsonl 2> gpurun_out/${TAG}_ab_cmp_1g.err || { echo "ab failed"; tail gpurun_out/${TAG}_ab_cmp_1g.err; exit 1; }
cat gpurun_out/${TAG}_ab_cmp_1g.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json 2> gpurun_out/${TAG}_bench_k20.err || { echo "bench k20 failed"; tail -20 gpurun_out/${TAG}_bench_k20.err; exit 1; }
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j[\"roofline\"]; print(\"k20\", j[\"value\"], r[\"avg_launch_us\"], r[\"frac\"], r[\"frac_of_achievable_per_block\"], j[\"barriered\"][\"frac\"], j[\"compute\"][\"overlapped\"][\"frac_vs_verify\"])" gpurun_out/${TAG}_bench_k20.json
