#!/bin/bash
# Round 4: config 5 in full (tools/e2e_read.py: host API, hdfsRead, 8 hdfsPreads, read-ahead 1/2/3/7
# and the short-circuit readers), one untimed pass per read-ahead / short-circuit line, 5 timed
# passes, the pool's retained pinned bytes under the default 1 GiB cap; twice.
set -o pipefail
TAG=${1:-r4u}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 400 python -u tools/e2e_read.py --reps 5 > gpurun_out/${TAG}_e2e_$i.jsonl 2> gpurun_out/${TAG}_e2e_$i.err \
    || { echo "e2e $i failed"; tail gpurun_out/${TAG}_e2e_$i.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/${TAG}_e2e_$i.jsonl'):
    d = json.loads(l); print(d['mode'], d.get('verify'), d.get('streams'), d.get('readahead_blocks'), d.get('gib_s'), d.get('gib_s_median'), d.get('gib_s_all'), d.get('cold_gib_s'), d.get('pool_retained_pinned_mib'))"
done
