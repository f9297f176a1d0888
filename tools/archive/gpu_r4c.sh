#!/bin/bash
# Round 4: the driver's-form ramp (tools/clock_ramp.py: per-launch shader clock from in-kernel
# stamps, lab variant 125) and the packet-stream solo last step (lab variant 124, tools/pkt_ab.py),
# after the parity tests of both variants.
set -o pipefail
TAG=${1:-r4c}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_packet_stream.py tests/test_gpu_parity.py -m gpu -q \
    -k "solo_variant or variants_overlapped" --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.txt | head; exit $rc; }
timeout -k 10 300 python -u tools/clock_ramp.py --reps 2 > gpurun_out/${TAG}_clock_ramp.jsonl 2> gpurun_out/${TAG}_clock_ramp.err
rc=$?; echo "clock_ramp rc=$rc"; cat gpurun_out/${TAG}_clock_ramp.jsonl; [ $rc -eq 0 ] || { tail gpurun_out/${TAG}_clock_ramp.err; exit $rc; }
for o in "" "--overlap"; do
  timeout -k 10 300 python -u tools/pkt_ab.py --variants 0,124 --rounds 7 $o > gpurun_out/${TAG}_pkt_ab$o.jsonl \
      2> gpurun_out/${TAG}_pkt_ab$o.err || { echo "pkt_ab $o failed"; tail gpurun_out/${TAG}_pkt_ab$o.err; exit 1; }
  cat gpurun_out/${TAG}_pkt_ab$o.jsonl
done
timeout -k 10 300 python -u tools/pkt_ab.py --variants 0,124 --rounds 5 --overlap --pitch 69632 \
    > gpurun_out/${TAG}_pkt_ab_aligned.jsonl 2> gpurun_out/${TAG}_pkt_ab_aligned.err && cat gpurun_out/${TAG}_pkt_ab_aligned.jsonl
