#!/bin/bash
# Round-3 pass: segment descriptors through the constant address space (s_load) instead of FLAT
# loads. -m gpu suite, then the segmented-kernel A/B (tools/seg_ab.py), the packet-stream rates
# and the batch API A/B, then the bench line.
set -o pipefail
TAG=${1:-r3j}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/seg_ab.py > gpurun_out/${TAG}_seg_ab.jsonl 2> gpurun_out/${TAG}_seg_ab.err \
    || { echo "seg_ab failed"; tail gpurun_out/${TAG}_seg_ab.err; exit 1; }
cat gpurun_out/${TAG}_seg_ab.jsonl
timeout -k 10 200 python -u tools/packets_rate.py > gpurun_out/${TAG}_packets_rate.jsonl 2> gpurun_out/${TAG}_packets_rate.err \
    || { echo "packets_rate failed"; tail gpurun_out/${TAG}_packets_rate.err; exit 1; }
cat gpurun_out/${TAG}_packets_rate.jsonl
timeout -k 10 200 python -u tools/batch_ab.py > gpurun_out/${TAG}_batch_ab.jsonl 2> gpurun_out/${TAG}_batch_ab.err \
    || { echo "batch_ab failed"; tail gpurun_out/${TAG}_batch_ab.err; exit 1; }
cat gpurun_out/${TAG}_batch_ab.jsonl
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j[\"roofline\"]; print(\"k2000\", j[\"value\"], r[\"avg_launch_us\"], r[\"frac\"], r[\"frac_of_achievable_per_block\"], j[\"barriered\"][\"frac\"], j[\"barriered\"][\"frac_of_achievable_per_block\"], j[\"batched\"][\"frac\"], j[\"compute\"][\"overlapped\"], j[\"compute\"][\"barriered\"][\"frac_vs_verify\"])" gpurun_out/${TAG}_bench.json
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json 2> gpurun_out/${TAG}_bench_k20.err \
    || { echo "bench k20 failed"; tail -20 gpurun_out/${TAG}_bench_k20.err; exit 1; }
python3 -c "import json,sys; j=json.load(open(sys.argv[1])); r=j[\"roofline\"]; print(\"k20\", j[\"value\"], r[\"avg_launch_us\"], r[\"frac\"], r[\"frac_of_achievable_per_block\"], j[\"barriered\"][\"frac\"], j[\"compute\"][\"overlapped\"][\"frac_vs_verify\"])" gpurun_out/${TAG}_bench_k20.json
