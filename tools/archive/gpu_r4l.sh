#!/bin/bash
# Round 4: every wave's start/end (launch-numbered slots) of 128 MiB verify and read launches,
# barriered and overlapped; the local-reader and host-API tests with streaming-store copies
# (HDFS3_COPY_NT=1); config 5 short-circuit reads with and without them (blocking window events).
set -o pipefail
TAG=${1:-r4l}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/wave_spread.py --k 40 > gpurun_out/${TAG}_spread.jsonl 2> gpurun_out/${TAG}_spread.err
rc=$?; echo "spread rc=$rc"; cat gpurun_out/${TAG}_spread.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_spread.err; exit $rc; }
HDFS3_COPY_NT=1 timeout -k 10 400 python -u -m pytest tests/test_local_reader.py tests/test_gpu_crc32.py -m gpu -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_nt_tests.txt 2>&1
rc=$?; echo "nt tests rc=$rc"; tail -2 gpurun_out/${TAG}_nt_tests.txt; [ $rc -eq 0 ] || exit $rc
for nt in 0 1 0 1; do
  HDFS3_COPY_NT=$nt HDFS3_LOCAL_BLOCKING_SYNC=1 timeout -k 10 300 python -u tools/e2e_read.py --local-only --reps 7 \
      >> gpurun_out/${TAG}_local_nt$nt.jsonl 2>> gpurun_out/${TAG}_local_nt$nt.err || { echo "local nt=$nt failed"; exit 1; }
done
for nt in 0 1; do echo "nt=$nt"; grep -E "local_read|host_verify" gpurun_out/${TAG}_local_nt$nt.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  ', d['mode'], d.get('verify'), d.get('streams'), d.get('gib_s_median', d.get('gib_s')), d.get('gib_s_all'))"; done
