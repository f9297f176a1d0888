#!/bin/bash
# Round 4, config 5: short-circuit readers (tools/e2e_read.py --local-only) with the copy pool's
# helper count 0 / 3 (default) / 8, and blocking window events (HDFS3_LOCAL_BLOCKING_SYNC=1);
# three repetitions each, every repetition reported.
set -o pipefail
TAG=${1:-r4j}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "3 0" "0 0" "8 0" "3 1" "8 1"; do
  set -- $cfg
  HDFS3_COPY_HELPERS=$1 HDFS3_LOCAL_BLOCKING_SYNC=$2 timeout -k 10 300 python -u tools/e2e_read.py --local-only --reps 3 \
      > gpurun_out/${TAG}_local_h$1_b$2.jsonl 2> gpurun_out/${TAG}_local_h$1_b$2.err || { echo "local $cfg failed"; exit 1; }
  echo "helpers=$1 blocking=$2"; grep -v plain_file gpurun_out/${TAG}_local_h$1_b$2.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  ', d['verify'], d['streams'], d['gib_s_all'])"
done
