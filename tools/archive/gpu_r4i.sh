#!/bin/bash
# Round 4: the build with size-based workgroups for verify: the full -m gpu suite, smoke(), the
# driver's bench form, and the A/B against 1024-thread workgroups everywhere (lab 137).
set -o pipefail
TAG=${1:-r4i}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.txt | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 \
    || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_k20.json \
    2> gpurun_out/${TAG}_bench_k20.err || { echo "bench k20 failed"; tail gpurun_out/${TAG}_bench_k20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_k20.json')); print('value', d['value'], d['roofline']['frac'], d['roofline'].get('frac_of_achievable_same_form'), 'bar', d['barriered']['frac'], d['barriered'].get('frac_of_achievable_per_block')); print('packets', d['packets']['overlapped']['frac_vs_contiguous'], d['packets']['barriered']['frac_vs_contiguous']); print('compute', d['compute']['overlapped']['frac_vs_verify'], d['compute']['overlapped']['paired']['compute_vs_verify'], d['compute']['barriered']['frac_vs_verify'], d['compute']['barriered']['paired']['compute_vs_verify']); print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['wall_s'])"
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run bar_4 --variants 0,137 --rounds 5 --block-mib 4 --blocks 128 --reps 100 &&
run bar_32 --variants 0,137 --rounds 5 --block-mib 32 --blocks 16 --reps 100 &&
run ovl_64 --variants 0,137 --rounds 5 --block-mib 64 --blocks 8 --reps 100 --overlap
timeout -k 10 300 python -u tools/pkt_ab.py --product --npk 64 --reps 400 --rounds 5 \
    > gpurun_out/${TAG}_pkt_4mib_bar.jsonl 2> gpurun_out/${TAG}_pkt_4mib_bar.err && cat gpurun_out/${TAG}_pkt_4mib_bar.jsonl
