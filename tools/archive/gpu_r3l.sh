#!/bin/bash
# Round-3 diagnostics: what the LDS table fill and the table math cost per 128 MiB launch
# (77 no math, 78 no math + no fill, 79 no fill; all wrong results on purpose), overlapped and
# barriered; then the bench's batch pass with its longer warmup.
set -o pipefail
TAG=${1:-r3l}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab.py --variants 0,77,78,79 --bpc 512,4096 --overlap --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_diag_ovl.jsonl 2> gpurun_out/${TAG}_ab_diag_ovl.err || { echo "ab failed"; tail gpurun_out/${TAG}_ab_diag_ovl.err; exit 1; }
cat gpurun_out/${TAG}_ab_diag_ovl.jsonl
timeout -k 10 300 python -u tools/ab.py --variants 0,77,78,79 --bpc 512 --rounds 15 --reps 100 \
    > gpurun_out/${TAG}_ab_diag_bar.jsonl 2> gpurun_out/${TAG}_ab_diag_bar.err || { echo "ab failed"; tail gpurun_out/${TAG}_ab_diag_bar.err; exit 1; }
cat gpurun_out/${TAG}_ab_diag_bar.jsonl
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j[\"roofline\"]; print(\"k2000\", j[\"value\"], r[\"avg_launch_us\"], r[\"frac\"], r[\"frac_of_achievable_per_block\"], j[\"barriered\"][\"frac\"], j[\"batched\"][\"avg_launch_us\"], j[\"batched\"][\"frac\"])" gpurun_out/${TAG}_bench.json
