#!/bin/bash
# Config 5 read lines under the round-3 host-side switches: NUMA placement (HDFS3_NUMA=0 turns it
# off) and the context pool's pinned cap (HDFS3_POOL_PINNED_MAX), interleaved twice.
set -o pipefail
TAG=${1:-r3e2eab}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() { # name env...
    local n=$1; shift
    env "$@" timeout -k 10 300 python -u tools/e2e_read.py --reps 2 --readahead 1,2,7 > gpurun_out/${TAG}_$n.jsonl 2> gpurun_out/${TAG}_$n.err \
        || { echo "e2e $n failed"; tail -20 gpurun_out/${TAG}_$n.err; exit 1; }
    echo "== $n"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    j=json.loads(l)
    if j['mode'].startswith('hdfsRead') or j['mode']=='parallel_pread': print(j['mode'], j.get('verify'), j.get('readahead_blocks',''), j['gib_s'])" gpurun_out/${TAG}_$n.jsonl
}
for rep in 1 2; do
run default_$rep HDFS3_E2E_TAG=default || exit 1
run nonuma_$rep HDFS3_NUMA=0 || exit 1
run bigcap_$rep HDFS3_POOL_PINNED_MAX=16G || exit 1
run both_$rep HDFS3_NUMA=0 HDFS3_POOL_PINNED_MAX=16G || exit 1
done
