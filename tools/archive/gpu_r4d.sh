#!/bin/bash
# Round 4: the full -m gpu suite and smoke() on the build with the packet-stream solo last step, the
# driver's bench form, the clock/timing of verify vs compute vs read regions (tools/clock_ramp.py),
# and packet-stream compute against contiguous compute (tools/pkt_ab.py --mode compute).
set -o pipefail
TAG=${1:-r4d}
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
cat gpurun_out/${TAG}_bench_k20.json
timeout -k 10 300 python -u tools/clock_ramp.py --reps 2 --kinds crc,compute,read --phases bench,steady \
    > gpurun_out/${TAG}_clock_ramp.jsonl 2> gpurun_out/${TAG}_clock_ramp.err
rc=$?; echo "clock_ramp rc=$rc"; cat gpurun_out/${TAG}_clock_ramp.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pkt_ab.py --variants 0 --rounds 5 --mode compute > gpurun_out/${TAG}_pkt_cmp.jsonl \
    2> gpurun_out/${TAG}_pkt_cmp.err && cat gpurun_out/${TAG}_pkt_cmp.jsonl
