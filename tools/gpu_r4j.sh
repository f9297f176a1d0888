#!/bin/bash
# Round 4, config 5: short-circuit readers (tools/e2e_read.py --local-only) with the copy pool's
# helper count 3 (default) / 8 / 12, three repetitions each, every repetition reported.
set -o pipefail
TAG=${1:-r4j}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for h in 0 3 8; do
  HDFS3_COPY_HELPERS=$h timeout -k 10 300 python -u tools/e2e_read.py --local-only --reps 3 \
      > gpurun_out/${TAG}_local_h$h.jsonl 2> gpurun_out/${TAG}_local_h$h.err || { echo "local h=$h failed"; exit 1; }
  echo "helpers=$h"; cat gpurun_out/${TAG}_local_h$h.jsonl
done
