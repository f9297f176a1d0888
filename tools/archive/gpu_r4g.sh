#!/bin/bash
# Round 4: staged compute words through system-scope nt stores (production) against plain stores
# (lab 128); 256-thread workgroups for small launches (lab 132) at the block reader's 4 MiB batch;
# the driver's bench form.
set -o pipefail
TAG=${1:-r4g}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_packet_stream.py -m gpu -q \
    -k "variants_overlapped or staged_words or solo_variant" --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.txt | head; exit $rc; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run cmp_ovl --variants 0,128 --rounds 11 --overlap --mode compute &&
run cmp_bar --variants 0,128 --rounds 7 --mode compute &&
run small_bar --variants 0,132 --rounds 7 --block-mib 4 --blocks 64 --reps 200 &&
run small_ovl --variants 0,132 --rounds 7 --block-mib 4 --blocks 64 --reps 200 --overlap &&
run mid_bar --variants 0,132 --rounds 5 --block-mib 16 --blocks 16 --reps 100 || exit 1
timeout -k 10 300 python -u tools/pkt_ab.py --variants 0,132 --npk 64 --reps 400 --rounds 5 \
    > gpurun_out/${TAG}_pkt_4mib_bar.jsonl 2> gpurun_out/${TAG}_pkt_4mib_bar.err && cat gpurun_out/${TAG}_pkt_4mib_bar.jsonl || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc \
    > gpurun_out/${TAG}_bench_k20.json 2> gpurun_out/${TAG}_bench_k20.err || { echo "bench failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_k20.json')); print('value', d['value'], d['roofline']['frac'], d['roofline'].get('frac_of_achievable_same_form'), 'bar', d['barriered']['frac'], d['barriered'].get('frac_of_achievable_per_block')); print('packets', d['packets']['overlapped']['frac_vs_contiguous'], d['packets']['barriered']['frac_vs_contiguous']); print('compute', d['compute']['overlapped']['frac_vs_verify'], d['compute']['overlapped']['paired']['compute_vs_verify'], d['compute']['barriered']['frac_vs_verify'], d['compute']['barriered']['paired']['compute_vs_verify'])"
