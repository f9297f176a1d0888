#!/bin/bash
# Config 5 rates with and without the copy pool's helper threads, same box, same call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for h in 3 0 3; do
  HDFS3_COPY_HELPERS=$h timeout -k 10 500 python -u tools/e2e_read.py --reps 2 > gpurun_out/ab_h${h}_$RANDOM.jsonl 2>/dev/null || exit 1
done
for f in gpurun_out/ab_h*.jsonl; do echo "== $f"; cut -c40-170 $f; done
