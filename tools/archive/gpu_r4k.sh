#!/bin/bash
# Round 4: every wave's start/end of 128 MiB verify and read launches, barriered and overlapped
# (tools/wave_spread.py): where the barriered launch's extra microseconds go.
set -o pipefail
TAG=${1:-r4k}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/wave_spread.py --k 40 > gpurun_out/${TAG}_spread.jsonl 2> gpurun_out/${TAG}_spread.err
rc=$?; echo "spread rc=$rc"; cat gpurun_out/${TAG}_spread.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_spread.err; exit $rc; }
timeout -k 10 300 python -u tools/wave_spread.py --k 40 --read-grid -256 --kinds read > gpurun_out/${TAG}_spread_r256.jsonl \
    2> gpurun_out/${TAG}_spread_r256.err && cat gpurun_out/${TAG}_spread_r256.jsonl
for b in 0 1 0 1; do
  HDFS3_LOCAL_BLOCKING_SYNC=$b timeout -k 10 300 python -u tools/e2e_read.py --local-only --reps 7 \
      >> gpurun_out/${TAG}_local_b$b.jsonl 2>> gpurun_out/${TAG}_local_b$b.err || { echo "local b=$b failed"; exit 1; }
done
for b in 0 1; do echo "blocking=$b"; grep local_read gpurun_out/${TAG}_local_b$b.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  ', d['verify'], d['streams'], d['gib_s_median'], d['gib_s_all'], d['cold_gib_s'])"; done
