#!/bin/bash
# Round 4: workgroup size by launch size (lab 132 = 256 threads, 134 = 512) from 4 MiB to 128 MiB,
# barriered and overlapped, HBM-resident block sets (>= 512 MiB rotated) and the block reader's
# cache-resident 64-packet batches; held compute words as system-scope nt stores at 1 GiB (lab 133).
set -o pipefail
TAG=${1:-r4h}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "variants_overlapped" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -1 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.txt | head; exit $rc; }
run() { local name=$1; shift
  timeout -k 10 300 python -u tools/ab.py "$@" > gpurun_out/${TAG}_${name}.jsonl 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/${TAG}_${name}.jsonl; return $rc; }
for mib in 4 16 32 64; do
  nb=$(( 512 / mib ))
  run bar_${mib} --variants 0,132,134 --rounds 5 --block-mib $mib --blocks $nb --reps 100 &&
  run ovl_${mib} --variants 0,132,134 --rounds 5 --block-mib $mib --blocks $nb --reps 100 --overlap || exit 1
done
run bar_128 --variants 0,132,134 --rounds 5 --reps 50 &&
run ovl_128 --variants 0,132,134 --rounds 5 --reps 50 --overlap || exit 1
timeout -k 10 300 python -u tools/pkt_ab.py --variants 0,132,134 --npk 64 --reps 400 --rounds 5 \
    > gpurun_out/${TAG}_pkt_4mib_bar.jsonl 2> gpurun_out/${TAG}_pkt_4mib_bar.err && cat gpurun_out/${TAG}_pkt_4mib_bar.jsonl || exit 1
run cmp_1g --variants 0,133 --rounds 5 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap --mode compute &&
run cmp_1g_4096 --variants 0,133 --rounds 5 --block-mib 1024 --blocks 2 --reps 8 --warm 200 --overlap --mode compute --bpc 4096 &&
run grid_short --variants 0,135,136 --rounds 9 --reps 20 --overlap &&
run grid_long --variants 0,135,136 --rounds 5 --reps 200 --overlap &&
run grid_bar --variants 0,135,136 --rounds 5 --reps 50
