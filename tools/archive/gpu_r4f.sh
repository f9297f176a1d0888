#!/bin/bash
# Round 4: the bench's packets block against tools/pkt_ab.py on one box (product library, the bench's
# region form), small launches (64 packets = 4 MiB, the block reader's batch) barriered, and the
# staged-word store policy (lab 128: system scope + nt) against production, more rounds.
set -o pipefail
TAG=${1:-r4f}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc \
    > gpurun_out/${TAG}_bench_k20.json 2> gpurun_out/${TAG}_bench_k20.err || { echo "bench failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_k20.json')); print('value', d['value'], d['roofline']['frac'], d['roofline'].get('frac_of_achievable_same_form')); print('packets', json.dumps(d['packets']['overlapped']['paired']), d['packets']['overlapped']['frac_vs_contiguous']); print('compute', json.dumps(d['compute']['overlapped']['paired']))"
timeout -k 10 300 python -u tools/pkt_ab.py --product --overlap --settle --warm-each 50 --reps 200 --rounds 3 \
    > gpurun_out/${TAG}_pkt_prod.jsonl 2> gpurun_out/${TAG}_pkt_prod.err && cat gpurun_out/${TAG}_pkt_prod.jsonl || exit 1
timeout -k 10 300 python -u tools/pkt_ab.py --variants 0,124 --overlap --rounds 5 \
    > gpurun_out/${TAG}_pkt_lab.jsonl 2> gpurun_out/${TAG}_pkt_lab.err && cat gpurun_out/${TAG}_pkt_lab.jsonl || exit 1
timeout -k 10 300 python -u tools/pkt_ab.py --product --npk 64 --reps 400 --rounds 5 \
    > gpurun_out/${TAG}_pkt_4mib_bar.jsonl 2> gpurun_out/${TAG}_pkt_4mib_bar.err && cat gpurun_out/${TAG}_pkt_4mib_bar.jsonl || exit 1
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
run cmp_ovl --variants 0,128,126,127 --rounds 11 --overlap --mode compute &&
run cmp_bar --variants 0,128 --rounds 7 --mode compute &&
run ver_ovl --variants 0 --rounds 11 --overlap --mode verify
